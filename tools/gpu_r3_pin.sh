#!/bin/bash
# Round 3: next-step operand loads pinned to the top of the k-step (SGP_GLOAD_PIN).  Parity on
# the new library (c), then alternating A/B against the previous one (b) for C3 VI, FITC,
# Laplace, C2 and the 8-GPU shard.  usage (inside gpurun): bash tools/gpu_r3_pin.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_c.so $L/libsgp.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],3), {k: p[k] for k in ('syrk','syrk_omega','contract_knm','rowquad_q','syrk_z','lap_obj') if k in p})"; }
for rep in 1 2; do
for v in b c; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/c3_$v$rep.json 2>/dev/null || { echo "c3 $v failed"; exit 1; }
  show $D/c3_$v$rep.json c3_$v$rep
  timeout -k 10 200 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc_$v$rep.json 2>/dev/null || { echo "fitc $v failed"; exit 1; }
  show $D/fitc_$v$rep.json fitc_$v$rep
  timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap_$v$rep.json 2>/dev/null || { echo "lap $v failed"; exit 1; }
  show $D/lap_$v$rep.json lap_$v$rep
  timeout -k 10 200 python3 bench.py --config C2 --steps 40 --warmup 3 --no-cpu-baseline > $D/c2_$v$rep.json 2>/dev/null || { echo "c2 $v failed"; exit 1; }
  show $D/c2_$v$rep.json c2_$v$rep
  timeout -k 10 200 python3 bench.py --rows 125000 --steps 20 --warmup 3 --no-cpu-baseline > $D/r125_$v$rep.json 2>/dev/null || { echo "r125 $v failed"; exit 1; }
  show $D/r125_$v$rep.json r125_$v$rep
done
done
cp $L/libsgp_c.so $L/libsgp.so
echo ok
