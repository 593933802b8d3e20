#!/bin/bash
# A/B of the contraction's rotated k order (SGP_CON_KROT): parity tests with it on, then
# alternating C2 / C3 / FITC bench runs.   usage (inside gpurun): bash tools/gpu_r3_krot.sh
set -o pipefail
D=gpurun_out/krot
mkdir -p $D
SGP_CON_KROT=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_fitc.py tests/test_gpu_sweep.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2 3; do for v in 0 1; do
  SGP_CON_KROT=$v timeout -k 10 100 python3 bench.py --config C2 --steps 40 --warmup 5 --no-cpu-baseline > $D/c2_$v$r.json 2> $D/c2_$v$r.err || exit 1
  SGP_CON_KROT=$v timeout -k 10 100 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $D/c3_$v$r.json 2> $D/c3_$v$r.err || exit 1
  echo "krot=$v run $r $(python3 -c "
import json
a=json.load(open('$D/c2_$v$r.json')); b=json.load(open('$D/c3_$v$r.json'))
print('C2', round(a['value'],1), 'con', round(a['phases_ms']['contract_knm'],4), ' C3', round(b['value'],3), 'con', round(b['phases_ms']['contract_knm'],3))")"
done; done
for v in 0 1; do
  SGP_CON_KROT=$v timeout -k 10 200 python3 bench.py --mode fitc --steps 4 --warmup 1 --no-cpu-baseline > $D/fitc_$v.json 2> $D/fitc_$v.err || exit 1
  echo "krot=$v fitc $(python3 -c "import json;d=json.load(open('$D/fitc_$v.json'));print(round(d['value'],3), {k: round(x,2) for k,x in d['phases_ms'].items()})")"
done
echo done
