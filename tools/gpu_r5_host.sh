# round 5: host-side share of a C2 evaluation -- plain C loop vs the Python paths
set -o pipefail
mkdir -p gpurun_out/host
for rep in 1 2; do
  timeout -k 10 120 ./tools/micro/eval_loop 100000 256 3 0 1000 || exit 1
  timeout -k 10 300 python3 tools/c2_loop.py C2 1000 || exit 1
done
timeout -k 10 300 python3 tools/host_overhead.py C2 - 300 || exit 1
