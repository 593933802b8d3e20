#!/bin/bash
# Round 3: Laplace NR part a as one K pass (k_lap_nr_a_fused) and grad_a's K x1 folded into the
# row-quadratic pass.  Parity on the new library (e), A/B against the previous one (d) on C5,
# and a kernel trace of the new one.  usage (inside gpurun): bash tools/gpu_r3_lap.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_e.so $L/libsgp.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['value'],3), round(d['ms_per_step'],3), d.get('nr_iterations', ''), d['phases_ms'])"; }
for rep in 1 2; do
for v in d e; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap_$v$rep.json 2>/dev/null || { echo "lap $v failed"; exit 1; }
  show $D/lap_$v$rep.json lap_$v$rep
done
done
cp $L/libsgp_e.so $L/libsgp.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/k -o run -- python3 bench.py --mode laplace --steps 5 --warmup 2 --no-cpu-baseline > $D/k.json 2> $D/k.err || { tail -20 $D/k.err; exit 1; }
echo ok
