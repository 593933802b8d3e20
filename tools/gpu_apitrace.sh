#!/bin/bash
# Host API + kernel timeline of the shard-size (n = 125k) and C2 evaluations: where does the
# host stall between launches?  usage: tools/gpu_apitrace.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $D/a125 -o run -- python3 bench.py --n 125000 --steps 5 --warmup 2 --no-cpu-baseline > $D/a125.json 2> $D/a125.err || { tail -20 $D/a125.err; exit 1; }
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
ls $D/a125 $D/c2
