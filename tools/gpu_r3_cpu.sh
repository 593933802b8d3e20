#!/bin/bash
# Round 3: SURVEY 8(d)'s full CPU plan on the box's CPU share, the default bench line (3-point
# CPU fit), and a kernel trace of C2 evaluations.  usage (inside gpurun): bash tools/gpu_r3_cpu.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
cat /sys/fs/cgroup/cpu.max > $D/cgroup_cpu_max.txt 2>&1; nproc >> $D/cgroup_cpu_max.txt; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> $D/cgroup_cpu_max.txt
timeout -k 10 500 python3 bench.py --cpu-full $D/cpu_full.json > $D/cpu_full.out 2> $D/cpu_full.err || { echo "cpu-full failed"; tail -20 $D/cpu_full.err; exit 1; }
timeout -k 10 300 python3 bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
cut -c1-300 $D/bench.json
cat $D/cgroup_cpu_max.txt
echo ok
