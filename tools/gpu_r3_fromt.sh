#!/bin/bash
# Round 3: FITC / Laplace gradient contractions from the two stored products in one pass
# (contract_pass_pair).  FITC / Laplace / knot / candidate / sweep / config parity, then C3 FITC
# and C5 Laplace A/B against the two-pass form (SGP_FROM_T_SEPARATE=1).
#   usage (inside gpurun): bash tools/gpu_r3_fromt.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest ${SGP_FROMT_TESTS:-tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_knots.py tests/test_gpu_candidates.py tests/test_gpu_objonly_candidates.py tests/test_gpu_sweep.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_drivers.py tests/test_mpmath.py} -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],4), d.get('objective'), {k: p[k] for k in ('contract_knm','contract_knm_b','lap_grad_b') if k in p})"; }
for rep in 1 2; do
  for v in sep fused; do
    E=""; [ $v = sep ] && E="SGP_FROM_T_SEPARATE=1"
    env $E timeout -k 10 200 python3 bench.py --mode fitc --steps 10 --warmup 2 --no-cpu-baseline > $D/fitc_$v$rep.json 2>$D/err || { echo "fitc $v failed"; tail -5 $D/err; exit 1; }
    show $D/fitc_$v$rep.json fitc_$v$rep
    env $E timeout -k 10 200 python3 bench.py --mode laplace --steps 20 --warmup 3 --no-cpu-baseline > $D/c5_$v$rep.json 2>$D/err || { echo "c5 $v failed"; tail -5 $D/err; exit 1; }
    show $D/c5_$v$rep.json c5_$v$rep
  done
done
echo ok
