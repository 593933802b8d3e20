# round 5: the column-layout GJ sweep -- micro-benchmark, parity subset, A/B (cur / oldsweep)
set -o pipefail
mkdir -p gpurun_out/gj
timeout -k 10 60 ./tools/micro/gj_sweep > gpurun_out/gj/sweep_micro.txt 2>&1 || { cat gpurun_out/gj/sweep_micro.txt; exit 1; }
cat gpurun_out/gj/sweep_micro.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_full.py > gpurun_out/gj/tests.log 2>&1 || { tail -30 gpurun_out/gj/tests.log; exit 1; }
tail -1 gpurun_out/gj/tests.log
bash tools/ab.sh gjc2 2 "oldsweep" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh gjsh 2 "oldsweep" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --devices 0 --steps 6 --warmup 2 > gpurun_out/gj/dev0_q8.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/gj/dev0_q8.json
