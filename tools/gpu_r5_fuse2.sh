# round 5: FITC / Laplace gradient passes over both stored products in one pass -- parity, A/B against r5h6
set -o pipefail
D=gpurun_out/fuse2
mkdir -p $D
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_tstore.py tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_multi.py \
  tests/test_gpu_knots.py tests/test_gpu_drivers.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
bash tools/ab.sh f2fitc 3 "r5h6" --mode fitc --steps 6 --warmup 2 || exit 1
bash tools/ab.sh f2c5 3 "r5h6" --config C5 --mode laplace --steps 10 --warmup 2 || exit 1
