# round 5: C2's t row sums on aux_lo in phase 2 (sgp_eval_vi only) -- parity, A/B against r5h5
set -o pipefail
D=gpurun_out/tdef
mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_multi.py \
  tests/test_gpu_knots.py tests/test_gpu_candidates.py tests/test_gpu_objonly_candidates.py tests/test_gpu_drivers.py tests/test_gpu_sweep.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
bash tools/ab.sh tdc2 4 "r5h5" --config C2 --steps 300 --warmup 20 || exit 1
