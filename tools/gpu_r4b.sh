set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4b/pytest.log; exit 1; }
tail -1 gpurun_out/r4b/pytest.log
bash tools/ab.sh r4b_c2 3 base --config C2 --steps 40 --warmup 3 && \
bash tools/ab.sh r4b_c3 2 base --steps 10 --warmup 2 && \
bash tools/ab.sh r4b_fitc 2 base --mode fitc --steps 8 --warmup 2 && \
bash tools/ab.sh r4b_lap 2 base --mode laplace --steps 10 --warmup 2
