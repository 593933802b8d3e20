#!/bin/bash
# Round 3: K22 chain without the copy blit and with its two tail launches fused.  Parity on the
# new library (b), C2 / C3 / C5 A/B against the previous one (a).
#   usage (inside gpurun): bash tools/gpu_r3_k22.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_b.so $L/libsgp.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],4), {k: p[k] for k in ('k22_aux','dense_bm','mm_vectors','contract_knm') if k in p})"; }
for rep in 1 2 3; do
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --config C2 --steps 60 --warmup 5 --no-cpu-baseline > $D/c2_$v$rep.json 2>/dev/null || { echo "c2 $v failed"; exit 1; }
  show $D/c2_$v$rep.json c2_$v$rep
done
done
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/c3_$v.json 2>/dev/null || { echo "c3 $v failed"; exit 1; }
  show $D/c3_$v.json c3_$v
  timeout -k 10 200 python3 bench.py --rows 125000 --steps 20 --warmup 3 --no-cpu-baseline > $D/r125_$v.json 2>/dev/null || { echo "r125 $v failed"; exit 1; }
  show $D/r125_$v.json r125_$v
done
cp $L/libsgp_b.so $L/libsgp.so
echo ok
