#!/bin/bash
# Round 3: share of the K12 builder run at reduced occupancy beside the K22 chain (FITC /
# Laplace phase 1), SGP_SHARED_SCALE x the modelled chain time; C5 Laplace and C3 FITC A/B.
#   usage (inside gpurun): bash tools/gpu_r3_shared.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],4), {k: p[k] for k in ('build_knm','k22_aux','rowquad_q') if k in p})"; }
for rep in 1 2; do
for sc in 1 0.5 0.25 0; do
  SGP_SHARED_SCALE=$sc timeout -k 10 200 python3 bench.py --mode laplace --steps 20 --warmup 3 --no-cpu-baseline > $D/c5_$sc.$rep.json 2>$D/err || { echo "c5 $sc failed"; tail -5 $D/err; exit 1; }
  show $D/c5_$sc.$rep.json c5_s$sc.$rep
done
done
for rep in 1 2; do
for sc in 1 0.5 0; do
  SGP_SHARED_SCALE=$sc timeout -k 10 200 python3 bench.py --mode fitc --steps 10 --warmup 2 --no-cpu-baseline > $D/fitc_$sc.$rep.json 2>$D/err || { echo "fitc $sc failed"; tail -5 $D/err; exit 1; }
  show $D/fitc_$sc.$rep.json fitc_s$sc.$rep
done
done
echo ok
