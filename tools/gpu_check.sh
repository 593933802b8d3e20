#!/bin/bash
# On the GPU box: GPU tests, one bench line, a kernel trace of a short bench run.
#   usage (inside gpurun): bash tools/gpu_check.sh TAG [extra bench args]
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo "bench failed"; tail -20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/$T/k.json 2> gpurun_out/$T/k.err || { echo "rocprof failed"; tail -20 gpurun_out/$T/k.err; exit 1; }
tail -1 gpurun_out/$T/pytest.log
echo ok
