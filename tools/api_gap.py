"""Host-gap view of a rocprofv3 --hip-trace --kernel-trace CSV pair (tools/gpu_apitrace.sh):
the kernels and HIP API calls of one evaluation, from the end of the previous evaluation's
gradient contraction to the end of this one's, with times relative to that end.
usage: python3 tools/api_gap.py DIR [EVAL_INDEX_FROM_END]"""
import csv
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
K = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
A = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K q" + k["Queue_Id"], k["Kernel_Name"][:64]) for k in K]
ev += [(int(a["Start_Timestamp"]), int(a["End_Timestamp"]), "A", a["Function"]) for a in A]
ev.sort()
cons = [e for e in ev if e[2].startswith("K") and "k_contract<" in e[3]]
c0, c1 = cons[-back - 1], cons[-back]
t0 = c0[1]
for e in ev:
    if t0 - 1 <= e[0] <= c1[0] + 1 or (e[2] == "A" and e[0] < t0 < e[1]):
        if e[2] == "A" and e[1] - e[0] < 1000 and "Launch" not in e[3] and "Memcpy" not in e[3] and "Synchron" not in e[3]:
            continue
        print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f} {e[2]:5s} {e[3]}")
print(f"eval span {(c1[1] - t0) / 1e3:.1f} us (contraction {(c1[1] - c1[0]) / 1e3:.1f} us)")
