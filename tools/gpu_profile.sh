#!/bin/bash
# The round's judged evidence, on the GPU box: GPU tests, the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace summary of the same command, separate FETCH_SIZE /
# WRITE_SIZE PMC passes for roofline.traffic, the secondary modes and per-rank shard sizes.
#   usage (inside gpurun): bash tools/gpu_profile.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
step() { echo "== $*"; }
step pytest
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
step bench
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/k.json 2> $D/k.err || { tail -20 $D/k.err; exit 1; }
step pmc-fetch
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pf -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/pf.json 2> $D/pf.err || { tail -20 $D/pf.err; exit 1; }
step pmc-write
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pw -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/pw.json 2> $D/pw.err || { tail -20 $D/pw.err; exit 1; }
step modes
timeout -k 10 300 python3 bench.py --mode fitc --steps 3 --warmup 1 --no-cpu-baseline > $D/fitc.json 2> $D/fitc.err || exit 1
timeout -k 10 300 python3 bench.py --mode laplace --steps 5 --warmup 2 --no-cpu-baseline > $D/laplace.json 2> $D/laplace.err || exit 1
step shards
for nn in 125000 250000 500000; do
  timeout -k 10 200 python3 bench.py --n $nn --steps 10 --warmup 3 --no-cpu-baseline > $D/rows$nn.json 2> $D/rows$nn.err || exit 1
done
tail -1 $D/pytest.log
echo ok
