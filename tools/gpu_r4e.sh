set -o pipefail
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4e/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4e/pytest.log; exit 1; }
tail -1 gpurun_out/r4e/pytest.log
bash tools/ab.sh r4e_c2 4 "base" --config C2 --steps 40 --warmup 3
