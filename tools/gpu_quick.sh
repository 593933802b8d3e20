#!/bin/bash
# Quick GPU check: a pytest subset and the C3 bench line (+ optional extra bench args).
#   usage (inside gpurun): bash tools/gpu_quick.sh TAG "pytest -k expr" ["extra bench args" ...]
set -o pipefail
T=$1; K=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
rc=$?
tail -n 6 $O/pytest.log
case $rc in 0|1|5) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -n 20 $O/bench_c3.err; exit 1; }
cut -c1-200 $O/bench_c3.json
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $a > $O/bench_x$i.json 2> $O/bench_x$i.err || { echo "bench $a failed"; tail -n 20 $O/bench_x$i.err; exit 1; }
done
python3 - "$O" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"], 3), d["ms_per_step"], d["phases_ms"])
PY
echo "pytest rc=$rc"
