#!/bin/bash
# Round 3: parity of the current library, then A/B of the FITC with-t SYRK variants
# (lib/libsgp_a.so = product, lib/libsgp_b.so = SGP_SYRK_T_EARLY=1), C2 / C3 lines and the C2
# host-issue profile.  usage (inside gpurun): bash tools/gpu_r3_ab.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_a.so $L/libsgp.so
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_edges.py tests/test_gpu_configs.py tests/test_rshim_exec.py tests/test_gpu_dist.py tests/test_gpu_knots.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc_$v$rep.json 2>/dev/null || { echo "fitc $v failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$D/fitc_$v$rep.json').read().strip().splitlines()[-1]); print('$v$rep', round(d['value'],3), d['phases_ms']['syrk'], d['phases_ms']['syrk_omega'])"
done
done
cp $L/libsgp_a.so $L/libsgp.so
timeout -k 10 200 python3 bench.py --config C2 --steps 40 --warmup 3 --no-cpu-baseline > $D/c2.json 2>/dev/null || { echo "c2 failed"; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/c3.json 2>/dev/null || { echo "c3 failed"; exit 1; }
timeout -k 10 200 python3 bench.py --n 125000 --steps 20 --warmup 3 --no-cpu-baseline > $D/r125.json 2>/dev/null || { echo "r125 failed"; exit 1; }
timeout -k 10 120 python3 tools/host_overhead.py C2 - 60 > $D/host_c2.txt 2>&1 || { echo "host failed"; exit 1; }
python3 - "$D" <<'PY'
import json, sys
for f in ("c2", "c3", "r125"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"], 3), round(d["ms_per_step"], 4), d["phases_ms"])
PY
cat $D/host_c2.txt
echo ok
