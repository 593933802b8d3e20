#!/bin/bash
# A/B timing on the GPU box: alternate the product library (lib/libsgp.so, "cur") with variant
# libraries built by `python -m sparsergps_amd._build variant NAME [REV] [-D...]` (loaded via
# SGP_AB_LIB; the product library is never overwritten).
#   usage (inside gpurun): bash tools/ab.sh TAG REPS "VARIANTS" BENCH_ARGS...
#   e.g.  bash tools/ab.sh c2syrk 3 "base" --config C2 --steps 40 --warmup 3
set -o pipefail
T=$1; REPS=$2; VARS=$3; shift 3
D=gpurun_out/$T
mkdir -p $D
for rep in $(seq 1 $REPS); do
  for v in cur $VARS; do
    # a variant is a library under tools/ab/, or env.VAR=VALUE: the product library with that
    # runtime switches, comma-separated (e.g. env.SGP_CON_SK=0)
    envset=""
    if [ "$v" = cur ]; then unset SGP_AB_LIB
    elif [ "${v#env.}" != "$v" ]; then unset SGP_AB_LIB; envset=$(echo "${v#env.}" | tr ',' ' ')
    else export SGP_AB_LIB=tools/ab/$v/libsgp.so; fi
    env $envset timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > $D/${v}_$rep.json 2> $D/${v}_$rep.err || { echo "bench $v failed"; tail -20 $D/${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$D/${v}_$rep.json')); print('$v', $rep, round(d['value'],2), round(d['ms_per_step'],4), {k: v for k, v in d['phases_ms'].items() if v > 0.01})"
  done
done
