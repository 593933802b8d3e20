#!/bin/bash
# Round-2 GPU check: all GPU tests, the plain bench line and the same bench under
# torch.distributed.run at N = 1 (RCCL collectives on the library stream).
#   usage (inside gpurun): bash tools/gpu_r2.sh TAG [pytest -k expr]
set -o pipefail
T=$1; K=${2:-}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=5 --timeout 420 --timeout-method thread "${KARG[@]}" > gpurun_out/$T/pytest.log 2>&1
rc=$?
tail -n 25 gpurun_out/$T/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -n 20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --no-cpu-baseline > gpurun_out/$T/bench_trun.json 2> gpurun_out/$T/bench_trun.err || { echo "torchrun bench failed"; tail -n 20 gpurun_out/$T/bench_trun.err; exit 1; }
cat gpurun_out/$T/bench.json gpurun_out/$T/bench_trun.json
echo "pytest rc=$rc"
