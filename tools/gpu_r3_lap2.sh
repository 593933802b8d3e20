#!/bin/bash
# Round 3: fused NR part a variants (e = first prefetching version, f = interleaved dot chains,
# h = f with a 128 KB row image), Laplace C5 A/B + parity of f.  usage: bash tools/gpu_r3_lap2.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_f.so $L/libsgp.so
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_laplace.py tests/test_gpu_configs.py tests/test_mpmath.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
for v in f h; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap_$v$rep.json 2>/dev/null || { echo "lap $v failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/lap_$v$rep.json').read().strip().splitlines()[-1]); print('$v$rep', round(d['value'],3), d['phases_ms']['lap_nr_a'])"
done
done
cp $L/libsgp_f.so $L/libsgp.so
echo ok
