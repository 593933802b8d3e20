# round 5: is C3's builder time thermal?  two runs back to back, a 90 s pause, a third run
set -o pipefail
D=gpurun_out/c3cool
mkdir -p $D
run() {
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/c3_$1.json 2> $D/c3_$1.err || { tail -20 $D/c3_$1.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$D/c3_$1.json') if l.startswith('{')][-1]; print('C3', '$1', round(d['value'], 3), {k: v for k, v in d['phases_ms'].items() if v > 1.0})"
}
run a && run b && echo "pause 90 s" && sleep 90 && run c
rocm-smi --showtemp --showpower 2>/dev/null | grep -i "card\|temp\|power" | head -8 || true
