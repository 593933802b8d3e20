set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for v in cur prev; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  timeout -k 10 120 python3 bench.py --n 125000 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/r125_$v$rep.json 2>/dev/null || exit 1
  timeout -k 10 120 python3 bench.py --config C2 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/ab/c2_$v$rep.json 2>/dev/null || exit 1
  echo "$v $rep $(python3 -c "import json;print(round(json.load(open('gpurun_out/ab/r125_$v$rep.json'))['ms_per_step'],3), round(json.load(open('gpurun_out/ab/c2_$v$rep.json'))['ms_per_step'],3))")"
done
done
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
timeout -k 10 120 ./tools/micro/kloop > gpurun_out/ab/kloop.txt 2>&1 && cat gpurun_out/ab/kloop.txt
