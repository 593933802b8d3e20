set -o pipefail
mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4k/pytest.log; exit 1; }
tail -1 gpurun_out/r4k/pytest.log
bash tools/ab.sh r4k_c3 2 base --steps 10 --warmup 2
