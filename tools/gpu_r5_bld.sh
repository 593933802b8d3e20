# round 5: VI builder with t in LDS (4 workgroups per CU) -- parity subset, A/B against HEAD~ (regbld)
set -o pipefail
mkdir -p gpurun_out/bld
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_knots.py tests/test_gpu_sweep.py > gpurun_out/bld/tests.log 2>&1 || { tail -30 gpurun_out/bld/tests.log; exit 1; }
tail -1 gpurun_out/bld/tests.log
bash tools/ab.sh bldc3 3 "regbld" --steps 10 --warmup 2 || exit 1
bash tools/ab.sh bldc2 2 "regbld" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh bldsh 2 "regbld" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
