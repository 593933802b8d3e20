#!/bin/bash
# Contraction epilogue K stages: inline-asm LDS-DMA (no compiler vmcnt(0) after each issue),
# triple-buffered two ahead.  Parity tests, per-tile stamps, then previous / current library
# on C2, C3, FITC and C5.   usage (inside gpurun): bash tools/gpu_r3_dma.sh
set -o pipefail
D=gpurun_out/dma
mkdir -p $D
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_sweep.py tests/test_gpu_edges.py tests/test_gpu_knots.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 60 ./tools/micro/con_trace $D/con_c2.csv 100000 256 > $D/con_c2.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/micro/con_trace $D/con_c3.csv 131072 1024 > $D/con_c3.txt 2>&1 || exit 1
tail -1 $D/con_c2.txt; tail -1 $D/con_c3.txt
for r in 1 2; do for v in prev cur; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  timeout -k 10 100 python3 bench.py --config C2 --steps 40 --warmup 5 --no-cpu-baseline > $D/c2_$v$r.json 2> $D/c2_$v$r.err || exit 1
  timeout -k 10 100 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > $D/c3_$v$r.json 2> $D/c3_$v$r.err || exit 1
  timeout -k 10 150 python3 bench.py --mode fitc --steps 4 --warmup 1 --no-cpu-baseline > $D/fitc_$v$r.json 2> $D/fitc_$v$r.err || exit 1
  timeout -k 10 150 python3 bench.py --mode laplace --steps 6 --warmup 2 --no-cpu-baseline > $D/lap_$v$r.json 2> $D/lap_$v$r.err || exit 1
  echo "$v run $r $(python3 -c "
import json
g=lambda f: json.load(open('$D/'+f+'_$v$r.json'))
a,b,c,l=g('c2'),g('c3'),g('fitc'),g('lap')
print('C2', round(a['value'],1), 'con', round(a['phases_ms']['contract_knm'],4), '| C3', round(b['value'],3), 'con', round(b['phases_ms']['contract_knm'],3), '| FITC', round(c['value'],3), '| C5', round(l['value'],2))")"
done; done
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
echo done
