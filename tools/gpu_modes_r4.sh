#!/bin/bash
# Round-4 closing pass: GPU suite on HEAD plus the secondary-mode bench lines and the C2 line.
#   usage (inside gpurun): bash tools/gpu_modes_r4.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=5 --timeout 420 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc.json 2> $D/fitc.err || exit 1
timeout -k 10 300 python3 bench.py --mode laplace --steps 10 --warmup 2 --no-cpu-baseline > $D/laplace.json 2> $D/laplace.err || exit 1
timeout -k 10 300 python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit 1
for f in fitc laplace c2 bench; do python3 -c "import json; d=json.loads(open('$D/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value'],3), round(d['ms_per_step'],3))"; done
echo "pytest rc=$rc"
