#!/bin/bash
# Matrix-core K12 builder for d up to 32: the whole GPU suite, then the previous (VALU builder
# for d > 8) and current library on C3-shaped runs at d = 8, 12, 20 (VI) and d = 12 (FITC).
#   usage (inside gpurun): bash tools/gpu_r3_bld.sh
set -o pipefail
D=gpurun_out/bld
mkdir -p $D
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
timeout -k 10 900 python3 -u -m pytest -q -m gpu --maxfail=3 --timeout 300 --timeout-method thread tests > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in prev cur; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  for dd in 8 12 20; do
    timeout -k 10 150 python3 bench.py --d $dd --steps 6 --warmup 2 --no-cpu-baseline > $D/vi$dd_$v.json 2> $D/vi${dd}_$v.err && mv $D/vi$dd_$v.json $D/vi${dd}_$v.json || { tail -20 $D/vi${dd}_$v.err; exit 1; }
    echo "$v vi d=$dd $(python3 -c "import json;d=json.load(open('$D/vi${dd}_$v.json'));print(round(d['value'],3), d['phases_ms'].get('build_knm'))")"
  done
  timeout -k 10 200 python3 bench.py --mode fitc --d 12 --steps 4 --warmup 1 --no-cpu-baseline > $D/fitc12_$v.json 2> $D/fitc12_$v.err || { tail -20 $D/fitc12_$v.err; exit 1; }
  echo "$v fitc d=12 $(python3 -c "import json;d=json.load(open('$D/fitc12_$v.json'));print(round(d['value'],3), d['phases_ms'].get('build_knm'))")"
done
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
echo done
