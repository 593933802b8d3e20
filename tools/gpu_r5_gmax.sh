# round 5: workgroups per persistent Gauss-Jordan chain (SGP_GJ_GMAX 128 = cur, 64, 192)
set -o pipefail
bash tools/ab.sh gmsh 2 "g64 g192" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
bash tools/ab.sh gmc2 2 "g64 g192" --config C2 --steps 300 --warmup 20 || exit 1
