#!/bin/bash
# Round-2 GPU pass: all GPU tests, then the bench lines (C3 headline, C2, C5 Laplace, FITC),
# then SURVEY 8(d)'s full CPU plan on the box's host (no GPU).
#   usage (inside gpurun): bash tools/gpu_r2b.sh TAG [pytest -k expr]
set -o pipefail
T=$1; K=${2:-}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=5 --timeout 420 --timeout-method thread "${KARG[@]}" > $O/pytest.log 2>&1
rc=$?
tail -n 25 $O/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench C3 failed"; tail -n 20 $O/bench_c3.err; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench C2 failed"; tail -n 20 $O/bench_c2.err; exit 1; }
timeout -k 10 300 python3 bench.py --mode laplace --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench C5 failed"; tail -n 20 $O/bench_c5.err; exit 1; }
timeout -k 10 300 python3 bench.py --mode fitc > $O/bench_fitc.json 2> $O/bench_fitc.err || { echo "bench FITC failed"; tail -n 20 $O/bench_fitc.err; exit 1; }
timeout -k 10 300 python3 bench.py --n 125000 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_rows125k.json 2> $O/bench_rows125k.err || { echo "bench rows failed"; tail -n 20 $O/bench_rows125k.err; exit 1; }
cat $O/bench_c3.json $O/bench_c2.json $O/bench_c5.json $O/bench_fitc.json $O/bench_rows125k.json | cut -c1-300
if [ "${SKIP_CPU_FULL:-0}" != 1 ]; then
  timeout -k 10 900 python3 bench.py --cpu-full $O/cpu_full.json > $O/cpu_full.out 2> $O/cpu_full.err || { echo "cpu-full failed"; tail -n 20 $O/cpu_full.err; exit 1; }
  tail -n 12 $O/cpu_full.err
fi
echo "pytest rc=$rc"
