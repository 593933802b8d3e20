set -o pipefail
mkdir -p gpurun_out/r4g
export TMPDIR=/tmp
true
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --rows 125000 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4g/trun125.json 2> gpurun_out/r4g/trun125.err || { tail -20 gpurun_out/r4g/trun125.err; exit 1; }
cut -c1-400 gpurun_out/r4g/trun125.json
timeout -k 10 300 python3 bench.py --rows 125000 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4g/plain125.json 2> gpurun_out/r4g/plain125.err && cut -c1-200 gpurun_out/r4g/plain125.json
