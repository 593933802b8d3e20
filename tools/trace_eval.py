#!/usr/bin/env python
"""Print the kernel timeline of the last full evaluation in a rocprofv3 kernel trace
(gaps between dispatches show host or launch overhead).

usage: python tools/trace_eval.py run_kernel_trace.csv [anchor-kernel-substring]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_contract<8, 0, false, false, false>"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("fewer than two anchor dispatches")
    a, b = idx[-2] + 1, idx[-1] + 1
    t0 = int(rows[a]["Start_Timestamp"])
    prev = None
    busy = 0
    for r in rows[a:b + 4]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e6:8.3f} ms  dur {(e - s) / 1e3:9.1f} us  gap {gap:8.1f} us  "
              f"q{r['Queue_Id']} {r['Kernel_Name'][:60]}")
        prev = e if prev is None else max(prev, e)
    t_end = int(rows[b]["End_Timestamp"])
    print(f"eval span {(t_end - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
