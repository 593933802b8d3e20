#!/bin/bash
# FITC / Laplace gradient passes over the stored products at d > 8 (k_contract<32, .., FROM_T>):
# parity tests, then FITC at C3's n, m with d = 12 on the previous (GEMM re-run) and the
# current library.   usage (inside gpurun): bash tools/gpu_r3_hd.sh
set -o pipefail
D=gpurun_out/hd
mkdir -p $D
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_sweep.py tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_knots.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for rep in 1 2; do for v in prev cur; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  timeout -k 10 200 python3 bench.py --mode fitc --d 12 --steps 4 --warmup 1 --no-cpu-baseline > $D/fitc12_$v$rep.json 2> $D/fitc12_$v$rep.err || { tail -20 $D/fitc12_$v$rep.err; exit 1; }
  echo "$v $rep $(cut -c1-150 $D/fitc12_$v$rep.json)"
done; done
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
echo done
