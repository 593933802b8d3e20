#!/bin/bash
# Round 3: row-quadratic epilogue with LDS-DMA staged K rows (b) against fragment-shaped global
# loads (a): parity of b, then FITC C3 and Laplace C5 A/B.  usage: bash tools/gpu_r3_rq.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_b.so $L/libsgp.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],3), {k: p[k] for k in ('rowquad_q','rowquad_p','lap_grad_a') if k in p})"; }
for rep in 1 2; do
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc_$v$rep.json 2>/dev/null || { echo "fitc $v failed"; exit 1; }
  show $D/fitc_$v$rep.json fitc_$v$rep
  timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap_$v$rep.json 2>/dev/null || { echo "lap $v failed"; exit 1; }
  show $D/lap_$v$rep.json lap_$v$rep
done
done
cp $L/libsgp_b.so $L/libsgp.so
echo ok
