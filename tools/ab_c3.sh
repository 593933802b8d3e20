#!/bin/bash
# A/B of builds of libsgp (sparsergps_amd/lib/libsgp_<variant>.so) on the C3 bench: value and
# the per-phase milliseconds, twice each, interleaved; the first variant is restored at the end.
# usage (inside gpurun): bash tools/ab_c3.sh VARIANT... (default: cur prev)
set -o pipefail
mkdir -p gpurun_out/ab3
V=${@:-cur prev}
for rep in 1 2; do
for v in $V; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab3/c3_$v$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab3/c3_$v$rep.json')); p=d['phases_ms']
print('$v $rep', round(d['value'],3), round(d['ms_per_step'],3), 'syrk', p.get('syrk'), 'con', p.get('contract_knm'), 'build', p.get('build_knm'))"
done
done
set -- $V
cp sparsergps_amd/lib/libsgp_$1.so sparsergps_amd/lib/libsgp.so
