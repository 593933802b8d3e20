# round 5: the split-K contraction tail -- parity subset, then A/B timings (cur / notail / r4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_sweep.py tests/test_gpu_fitc.py \
  tests/test_gpu_laplace.py tests/test_gpu_edges.py > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
bash tools/ab.sh c2tail 3 "notail r4" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh c3tail 2 "notail r4" --config C3 --steps 10 --warmup 2 || exit 1
bash tools/ab.sh shtail 2 "notail r4" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
