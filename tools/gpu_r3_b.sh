#!/bin/bash
# Round 3 batch: parity of the product build, torchrun shard line + LDS counters (gpu_r3_misc),
# a C2 kernel trace, and the Ozaki int8 experiment.  usage: bash tools/gpu_r3_b.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fitc.py tests/test_gpu_knots.py tests/test_gpu_laplace.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
bash tools/gpu_r3_misc.sh $T/misc || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
timeout -k 10 300 ./tools/micro/ozaki > $D/ozaki.txt 2>&1 || { echo "ozaki failed"; tail -20 $D/ozaki.txt; exit 1; }
cat $D/ozaki.txt
echo ok
