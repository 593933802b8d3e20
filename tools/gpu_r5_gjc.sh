# round 5: persistent GJ with the chain on one workgroup (P in LDS) -- parity, A/B against the pool-only version (gjpool)
set -o pipefail
mkdir -p gpurun_out/gjc
timeout -k 10 150 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_vi.py > gpurun_out/gjc/t_vi.log 2>&1 || { tail -40 gpurun_out/gjc/t_vi.log; exit 1; }
tail -1 gpurun_out/gjc/t_vi.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_fitc.py \
  tests/test_gpu_laplace.py tests/test_gpu_multi.py tests/test_gpu_full.py tests/test_gpu_predict.py tests/test_gpu_sweep.py > gpurun_out/gjc/tests.log 2>&1 || { tail -40 gpurun_out/gjc/tests.log; exit 1; }
tail -1 gpurun_out/gjc/tests.log
bash tools/ab.sh gjcc2 3 "gjpool gjsteps" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh gjcsh 2 "gjpool gjsteps" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
