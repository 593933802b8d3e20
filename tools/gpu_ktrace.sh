#!/bin/bash
# Kernel-only timelines (no API tracing, so launches are issued at their normal host cost) of
# the C2 and the n = 125k shard evaluations, for tools/idle_gaps.py.  usage: tools/gpu_ktrace.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/a125 -o run -- python3 bench.py --n 125000 --steps 5 --warmup 2 --no-cpu-baseline > $D/a125.json 2> $D/a125.err || { tail -20 $D/a125.err; exit 1; }
ls $D/c2 $D/a125
