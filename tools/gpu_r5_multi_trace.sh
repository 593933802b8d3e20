# round 5: kernel trace of the in-library one-shard RCCL path (C3) to locate its overhead
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mt/dev0 -o run -- python3 bench.py --devices 0 --steps 4 --warmup 1 > gpurun_out/mt/dev0.json 2> gpurun_out/mt/dev0.err || { tail -20 gpurun_out/mt/dev0.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mt/plain -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/mt/plain.json 2> gpurun_out/mt/plain.err || { tail -20 gpurun_out/mt/plain.err; exit 1; }
ls -R gpurun_out/mt | head -30
