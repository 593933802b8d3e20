# round 5: C2 -- K22 built on the main stream (cur) against on aux beside the SYRK (k22aux)
# m-vector scalars on aux_lo; parity, then A/B against r5h7 (HEAD before them)
set -o pipefail
D=gpurun_out/tail7
mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_multi.py \
  tests/test_gpu_knots.py tests/test_gpu_candidates.py tests/test_gpu_objonly_candidates.py tests/test_gpu_drivers.py tests/test_gpu_sweep.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
bash tools/ab.sh t7c2 4 "k22aux" --config C2 --steps 300 --warmup 20 || exit 1
