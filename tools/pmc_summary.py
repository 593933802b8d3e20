#!/usr/bin/env python
"""Per-kernel summary of a rocprofv3 --pmc counter CSV: mean counter values per dispatch for
the hot kernels, plus MFMA-busy fraction and effective clock where the counters allow.

usage: python tools/pmc_summary.py run_counter_collection.csv [kernel-substring ...]
"""
import collections
import csv
import sys

DEFAULT = ["k_contract<8, 0, false, false, false>", "k_syrk_blk", "k_build_knm<true, 8>"]
SIMDS = 1024   # 256 CUs x 4 SIMDs (MI355X)


def main():
    path = sys.argv[1]
    keys = sys.argv[2:] or DEFAULT
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        for k in keys:
            if k in r["Kernel_Name"]:
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                agg[k][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    for k, cs in agg.items():
        print(k)
        durs = None
        for c, xs in sorted(cs.items()):
            mean = sum(x for x, _ in xs) / len(xs)
            durs = [d for _, d in xs]
            print(f"   {c:28s} {mean:.4g}  (n={len(xs)})")
        dur = sum(durs) / len(durs) * 1e-9
        if "GRBM_GUI_ACTIVE" in cs:
            g = sum(x for x, _ in cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"])
            clk = g / 8 / dur
            print(f"   effective clock {clk / 1e9:.3f} GHz over {dur * 1e3:.2f} ms")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
                mb = sum(x for x, _ in cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
                print(f"   MFMA busy {mb / (SIMDS * dur * clk):.3f} of SIMD cycles")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
            bc = sum(x for x, _ in cs["SQ_LDS_BANK_CONFLICT"]) / len(cs["SQ_LDS_BANK_CONFLICT"])
            la = sum(x for x, _ in cs["SQ_LDS_IDX_ACTIVE"]) / len(cs["SQ_LDS_IDX_ACTIVE"])
            print(f"   LDS conflict cycles / LDS active cycles {bc / max(la, 1):.3f}")


if __name__ == "__main__":
    main()
