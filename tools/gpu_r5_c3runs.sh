# round 5: C3 (bench.py's default line) four times on one box, HEAD
set -o pipefail
D=gpurun_out/c3runs
mkdir -p $D
for r in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/c3_$r.json 2> $D/c3_$r.err || { tail -20 $D/c3_$r.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$D/c3_$r.json') if l.startswith('{')][-1]; print('C3', $r, round(d['value'], 3), round(d['ms_per_step'], 3), {k: v for k, v in d['phases_ms'].items() if v > 0.2})"
done
