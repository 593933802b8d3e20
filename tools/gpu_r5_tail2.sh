set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh c2tail 2 "notail r4" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh c3tail 2 "notail r4" --config C3 --steps 10 --warmup 2 || exit 1
bash tools/ab.sh shtail 2 "notail r4" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
