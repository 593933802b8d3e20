# round 5: lean ctypes path of SparseGPContext.eval_vi / eval_fitc -- parity, Python gap split
set -o pipefail
D=gpurun_out/pyfast
mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vi.py tests/test_gpu_fitc.py tests/test_gpu_configs.py tests/test_gpu_objonly_candidates.py tests/test_gpu_drivers.py tests/test_gpu_multi.py tests/test_gpu_tstore.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
SGP_AB_LIB=tools/ab/hprobe/libsgp.so timeout -k 10 200 python3 tools/c2_pygap.py 400
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --config C2 --steps 300 --warmup 20 > $D/c2_$r.json 2> $D/c2_$r.err || { tail -20 $D/c2_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/c2_$r.json')); print('C2', round(d['value'], 1))"
done
