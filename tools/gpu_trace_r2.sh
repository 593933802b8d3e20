#!/bin/bash
# Timelines: kernel trace of the shard-size (n = 125 000) evaluation and of C2; the per-tile
# phase stamps of the contraction (tools/micro/con_trace).
#   usage (inside gpurun): bash tools/gpu_trace_r2.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/k125 -o run -- python3 bench.py --n 125000 --steps 5 --warmup 2 --no-cpu-baseline > $D/k125.json 2> $D/k125.err || { tail -20 $D/k125.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/kc2 -o run -- python3 bench.py --config C2 --steps 5 --warmup 2 --no-cpu-baseline > $D/kc2.json 2> $D/kc2.err || { tail -20 $D/kc2.err; exit 1; }
timeout -k 10 120 ./tools/micro/con_trace $D/con_trace.csv > $D/con_trace.txt 2>&1 || { tail -5 $D/con_trace.txt; exit 1; }
cat $D/con_trace.txt
python3 tools/trace_eval.py $D/k125/run_kernel_trace.csv > $D/timeline125.txt && tail -45 $D/timeline125.txt
python3 tools/trace_eval.py $D/kc2/run_kernel_trace.csv > $D/timelinec2.txt && tail -5 $D/timelinec2.txt
