# round 5: host-side time of sgp_eval_vi at C2 and C3 (variant with SGP_HOST_PROBE)
set -o pipefail
D=gpurun_out/hprobe
mkdir -p $D
export SGP_AB_LIB=tools/ab/hprobe/libsgp.so
timeout -k 10 200 python3 bench.py --no-cpu-baseline --config C2 --steps 600 --warmup 20 > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
grep "host probe" $D/c2.err | tail -3
python3 -c "import json; d=json.load(open('$D/c2.json')); print('C2', d['value'])"
