set -o pipefail
mkdir -p gpurun_out/det
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_determinism.py tests/test_gpu_multi.py tests/test_gpu_fitc.py tests/test_gpu_laplace.py > gpurun_out/det/tests.log 2>&1 || { tail -30 gpurun_out/det/tests.log; exit 1; }
grep -E "passed|C4|candidates" gpurun_out/det/tests.log
for a in "--devices 0 --steps 10 --warmup 2" "--steps 10 --warmup 2 --no-cpu-baseline" "--devices 0,0,0,0,0,0,0,0 --steps 6 --warmup 2" "--config C2 --devices 0 --steps 300 --warmup 20" "--config C2 --steps 300 --warmup 20 --no-cpu-baseline"; do
  timeout -k 10 300 python3 bench.py $a > gpurun_out/det/run.json 2> gpurun_out/det/run.err || { tail -20 gpurun_out/det/run.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/det/run.json') if l.startswith('{')][-1]; print('$a', round(d['value'],2), round(d['ms_per_step'],3))"
done
