#!/bin/bash
# Round 3: builder -> SYRK pipeline in VI phase 1 (SGP_SYRK_PIPE).  VI parity with the pipeline
# forced on at every size, the headline-shape tests at the default, then C3 / shard A/B.
#   usage (inside gpurun): bash tools/gpu_r3_pipe.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
SGP_SYRK_PIPE=1 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_sweep.py tests/test_gpu_edges.py tests/test_gpu_knots.py tests/test_gpu_candidates.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread > $D/pytest_forced.log 2>&1 || { echo "forced pytest failed"; tail -30 $D/pytest_forced.log; exit 1; }
tail -1 $D/pytest_forced.log
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > $D/pytest_default.log 2>&1 || { echo "default pytest failed"; tail -30 $D/pytest_default.log; exit 1; }
tail -1 $D/pytest_default.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],4), {k: p[k] for k in ('build_knm','syrk','syrk_reduce','dense_bm','contract_knm') if k in p})"; }
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline $BARGS > $D/$name.json 2>$D/$name.err || { echo "$name failed"; tail -5 $D/$name.err; exit 1; }
  show $D/$name.json $name
}
BARGS="--steps 20 --warmup 3"
for rep in 1 2; do
  run c3_off$rep SGP_SYRK_PIPE=0
  run c3_on$rep SGP_SYRK_PIPE=1
  run c3_w1_$rep SGP_SYRK_PIPE=1 SGP_SYRK_PIPE_WPC=1
  run c3_w3_$rep SGP_SYRK_PIPE=1 SGP_SYRK_PIPE_WPC=3
  run c3_f25_$rep SGP_SYRK_PIPE=1 SGP_SYRK_PIPE_FRAC=0.25
done
BARGS="--n 125000 --steps 20 --warmup 3"
for rep in 1 2; do
  run r125_off$rep SGP_SYRK_PIPE=0
  run r125_on$rep SGP_SYRK_PIPE=1
  run r125_w1_$rep SGP_SYRK_PIPE=1 SGP_SYRK_PIPE_WPC=1
done
echo ok
