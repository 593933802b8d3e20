#!/usr/bin/env python
"""Turn two rocprofv3 --pmc counter CSVs (FETCH_SIZE pass, WRITE_SIZE pass) into the per-launch
HBM traffic record bench.py reports as roofline.traffic (profiles/pmc_traffic_contract_knm.json).

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): counters
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16 B/lane streaming loads, so it is
doubled; WRITE_SIZE is exact.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv --n 1000000 --m 1024 [--out JSON]
"""
from __future__ import annotations

import argparse
import csv
import json

KERNEL_MATCH = "k_contract<8, 0, false, false, false, true, false>"   # VI "contract_knm" (EPI_GRAD, GEMM k-loop)


def per_launch(path, counter, match):
    vals = []
    name = None
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or match not in row["Kernel_Name"]:
            continue
        vals.append(float(row["Counter_Value"]))
        name = row["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for kernels matching {match!r} in {path}")
    return sum(vals) / len(vals), len(vals), name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--m", type=int, required=True)
    ap.add_argument("--match", default=KERNEL_MATCH)
    ap.add_argument("--out", default="profiles/pmc_traffic_contract_knm.json")
    a = ap.parse_args()
    f_kib, nf, name = per_launch(a.fetch_csv, "FETCH_SIZE", a.match)
    w_kib, nw, _ = per_launch(a.write_csv, "WRITE_SIZE", a.match)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    # algorithmic: K12 read once (8 B/pair) + P (8 m^2 B) + row vectors/gradient slab (small)
    alg = 8.0 * a.n * a.m + 8.0 * a.m * a.m
    rec = {
        "kernel": name,
        "n": a.n, "m": a.m,
        "fetch_size_kib_raw": f_kib,
        "write_size_kib": w_kib,
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "correction": "FETCH_SIZE doubled (gfx950 reports half the bytes of 16 B/lane streaming "
                      "loads, MI355X_MICROARCH.md HBM section); WRITE_SIZE exact; KiB units",
        "source": [a.fetch_csv, a.write_csv],
        "launches": min(nf, nw),
    }
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
