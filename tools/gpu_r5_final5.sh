# round 5 closing: GPU suite on HEAD, default bench line, rocprofv3 kernel stats, mode lines
set -o pipefail
D=gpurun_out/r5final5
mkdir -p $D
timeout -k 10 1100 python -u -m pytest --maxfail=5 -v -s --timeout 300 --timeout-method thread -m gpu tests/ > $D/suite.log 2>&1 || { tail -30 $D/suite.log; exit 1; }
tail -1 $D/suite.log
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=[json.loads(l) for l in open('$D/bench.json') if l.startswith('{')][-1]; print('bench', round(d['value'],3), d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/k.json 2> $D/k.err || { tail -20 $D/k.err; exit 1; }
for a in "--config C2 --steps 300 --warmup 20" "--n 125000 --steps 40 --warmup 4" "--mode fitc --steps 6 --warmup 2" "--config C5 --mode laplace --steps 10 --warmup 2" "--knots --steps 6 --warmup 2"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $a > $D/run.json 2> $D/run.err || { tail -20 $D/run.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$D/run.json') if l.startswith('{')][-1]; print('$a', round(d['value'],2), round(d['ms_per_step'],3))"
  cp $D/run.json "$D/run_$(echo $a | tr -c 'a-zA-Z0-9' '_').json"
done
