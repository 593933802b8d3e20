#!/usr/bin/env python
"""Summarise tools/gpu_run.sh's builderpmc passes: per kernel (k_build_knm_mfma,
k_diag_store_tile) the mean duration and every counter, per launch, and the derived write-path
figures (GB/s, WRITE_SIZE vs the bytes stored, EA write latency = WRREQ_LEVEL / WRREQ, writes in
flight = WRREQ_LEVEL / cycles, VALU-active and VMEM-write-issue shares of the wave cycles).
usage: python tools/builder_pmc_summary.py gpurun_out/r6d [--out profiles/r6/builder_pmc.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"builder": "k_build_knm_mfma", "store_ceiling": "k_diag_store_tile"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    vals = {k: defaultdict(list) for k in KERNELS}
    durs = {k: {} for k in KERNELS}
    for path in sorted(glob.glob(os.path.join(a.dir, "bpmc_*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(path)):
            for key, match in KERNELS.items():
                if match in row["Kernel_Name"]:
                    vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    durs[key][(path, row["Dispatch_Id"])] = (int(row["End_Timestamp"]) -
                                                             int(row["Start_Timestamp"])) * 1e-9
    out = {}
    for key in KERNELS:
        v = {c: sum(x) / len(x) for c, x in vals[key].items()}
        d = list(durs[key].values())
        t = sum(d) / len(d) if d else float("nan")
        rec = {"kernel": KERNELS[key], "launches_profiled": len(d), "mean_duration_ms": t * 1e3,
               "counters_per_launch": v}
        if "WRITE_SIZE" in v:
            rec["write_bytes"] = v["WRITE_SIZE"] * 1024.0
            rec["write_gbs"] = rec["write_bytes"] / t / 1e9
        if "TCC_EA0_WRREQ_sum" in v and v.get("TCC_EA0_WRREQ_sum"):
            rec["ea_write_latency_cycles"] = v["TCC_EA0_WRREQ_LEVEL_sum"] / v["TCC_EA0_WRREQ_sum"]
        if "GRBM_GUI_ACTIVE" in v:
            clk = v["GRBM_GUI_ACTIVE"] / 8.0 / t     # GRBM counts per XCD (8), cycles per second
            rec["clock_ghz"] = clk / 1e9
            if "TCC_EA0_WRREQ_LEVEL_sum" in v:
                rec["ea_writes_in_flight"] = v["TCC_EA0_WRREQ_LEVEL_sum"] / (t * clk)
            if "SQ_WAVE_CYCLES" in v and v["SQ_WAVE_CYCLES"]:
                rec["valu_active_share"] = v["SQ_ACTIVE_INST_VALU"] / v["SQ_WAVE_CYCLES"]
                rec["vmem_wr_issue_share"] = v["SQ_INST_CYCLES_VMEM_WR"] / v["SQ_WAVE_CYCLES"]
                rec["wait_inst_any_share"] = v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"]
        out[key] = rec
    text = json.dumps(out, indent=1)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
