"""GPU idle intervals of one evaluation from a rocprofv3 --kernel-trace CSV: the union of all
queues' kernel intervals between two consecutive gradient contractions, and every gap in it
longer than 2 us with the kernels on either side.  usage: python3 tools/idle_gaps.py CSV [k]"""
import csv
import sys

K = list(csv.DictReader(open(sys.argv[1])))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ev = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:60]) for k in K)
cons = [e for e in ev if "k_contract<" in e[2]]
lo, hi = cons[-back - 1][1], cons[-back][1]
win = [e for e in ev if lo <= e[0] < hi]
busy_end, idle, last = lo, 0, cons[-back - 1]
for s, e, nm in win:
    if s > busy_end + 2000:
        print(f"  idle {(s - busy_end) / 1e3:7.1f} us at {(busy_end - lo) / 1e3:8.1f}: after {last[2][:40]:40s} before {nm[:40]}")
    if s > busy_end:
        idle += s - busy_end
    if e > busy_end:
        busy_end, last = e, (s, e, nm)
print(f"eval {(hi - lo) / 1e3:.1f} us, GPU idle {idle / 1e3:.1f} us, kernels {len(win)}")
