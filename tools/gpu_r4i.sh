set -o pipefail
mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4i/pytest.log; exit 1; }
tail -1 gpurun_out/r4i/pytest.log
bash tools/ab.sh r4i_fitc 2 base --mode fitc --steps 8 --warmup 2 && \
bash tools/ab.sh r4i_lap 3 base --mode laplace --steps 10 --warmup 2
