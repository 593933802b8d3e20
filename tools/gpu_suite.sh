set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest --maxfail=5 -v -s --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/suite.log 2>&1
