"""One line per bench JSON of a tools/ab.sh run (gpurun_out/<TAG>/<variant>_<rep>.json):
    python tools/ab_table.py TAG [TAG ...]   (phases above 0.01 ms)"""
import glob
import json
import os
import sys

for tag in sys.argv[1:]:
    for f in sorted(glob.glob(f"gpurun_out/{tag}/*.json")):
        d = json.load(open(f))
        ph = {k: round(v, 4) for k, v in d.get("phases_ms", {}).items() if v > 0.01}
        print(f"{tag} {os.path.basename(f)[:-5]} {d['value']:.2f} {d['ms_per_step']:.4f} {ph}")
