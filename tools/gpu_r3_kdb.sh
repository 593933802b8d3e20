#!/bin/bash
# A/B of the contraction epilogue's double-buffered half-height K stages (lib/libsgp_kdb.so,
# SGP_CON_KDB=1) against the product library (lib/libsgp_prod.so): parity of the KDB build on
# every gradient-epilogue test, then C3 / C2 / n = 125k lines, twice each.
#   usage (inside gpurun): bash tools/gpu_r3_kdb.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_kdb.so $L/libsgp.so
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fitc.py tests/test_gpu_knots.py tests/test_gpu_laplace.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_kdb.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest_kdb.log; cp $L/libsgp_prod.so $L/libsgp.so; exit 1; }
tail -1 $D/pytest_kdb.log
for rep in 1 2; do
for v in prod kdb; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/c3_$v$rep.json 2>/dev/null || { echo "c3 $v failed"; exit 1; }
  timeout -k 10 200 python3 bench.py --config C2 --steps 40 --warmup 3 --no-cpu-baseline > $D/c2_$v$rep.json 2>/dev/null || { echo "c2 $v failed"; exit 1; }
  python3 - "$D" "$v$rep" <<'PY'
import json, sys
d, tag = sys.argv[1], sys.argv[2]
a = json.loads(open(f"{d}/c3_{tag}.json").read().strip().splitlines()[-1])
b = json.loads(open(f"{d}/c2_{tag}.json").read().strip().splitlines()[-1])
print(tag, "c3", round(a["value"], 3), a["phases_ms"]["contract_knm"], "c2", round(b["value"], 1), b["phases_ms"]["contract_knm"])
PY
done
done
cp $L/libsgp_prod.so $L/libsgp.so
echo ok
