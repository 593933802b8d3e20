set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4c/pytest.log; exit 1; }
tail -1 gpurun_out/r4c/pytest.log
bash tools/ab.sh r4c_c2 3 "base notail" --config C2 --steps 40 --warmup 3 && \
bash tools/ab.sh r4c_r125 2 "base notail" --n 125000 --steps 10 --warmup 2 && \
bash tools/ab.sh r4c_c3 1 "base notail" --steps 10 --warmup 2
