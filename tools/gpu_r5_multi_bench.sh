# round 5: the in-library multi-device context timed (C4 composition on one GPU; one shard via RCCL)
set -o pipefail
mkdir -p gpurun_out/mb
timeout -k 10 300 python3 bench.py --devices 0,0,0,0,0,0,0,0 --steps 10 --warmup 2 > gpurun_out/mb/c4_shards8.json 2> gpurun_out/mb/c4_shards8.err || { tail -20 gpurun_out/mb/c4_shards8.err; exit 1; }
cat gpurun_out/mb/c4_shards8.json
timeout -k 10 300 python3 bench.py --devices 0 --steps 10 --warmup 2 > gpurun_out/mb/c3_dev0.json 2> gpurun_out/mb/c3_dev0.err || { tail -20 gpurun_out/mb/c3_dev0.err; exit 1; }
cat gpurun_out/mb/c3_dev0.json
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/mb/c3_plain.json 2> gpurun_out/mb/c3_plain.err || { tail -20 gpurun_out/mb/c3_plain.err; exit 1; }
cat gpurun_out/mb/c3_plain.json
timeout -k 10 300 python3 bench.py --n 125000 --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/mb/shard_plain.json 2> gpurun_out/mb/shard_plain.err || { tail -20 gpurun_out/mb/shard_plain.err; exit 1; }
cat gpurun_out/mb/shard_plain.json
timeout -k 10 300 python3 bench.py --mode fitc --devices 0,0,0,0,0,0,0,0 --steps 4 --warmup 1 > gpurun_out/mb/fitc_shards8.json 2> gpurun_out/mb/fitc_shards8.err || { tail -20 gpurun_out/mb/fitc_shards8.err; exit 1; }
cat gpurun_out/mb/fitc_shards8.json
timeout -k 10 300 python3 bench.py --mode laplace --devices 0,0,0,0 --steps 5 --warmup 2 > gpurun_out/mb/lap_shards4.json 2> gpurun_out/mb/lap_shards4.err || { tail -20 gpurun_out/mb/lap_shards4.err; exit 1; }
cat gpurun_out/mb/lap_shards4.json
