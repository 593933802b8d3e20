#!/bin/bash
# Round 3: square-root staging of the weighted SYRK rows (k_syrk_blk wsqrt).  Parity on the new
# library (b), then alternating A/B against the previous one (a): FITC C3, Laplace C5, C3 VI.
#   usage (inside gpurun): bash tools/gpu_r3_sq.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_b.so $L/libsgp.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
show() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d.get('phases_ms',{}); print('$2', round(d['value'],3), round(d['ms_per_step'],3), {k: p[k] for k in ('syrk','syrk_omega','syrk_z','lap_obj','contract_knm') if k in p})"; }
for rep in 1 2; do
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc_$v$rep.json 2>/dev/null || { echo "fitc $v failed"; exit 1; }
  show $D/fitc_$v$rep.json fitc_$v$rep
  timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap_$v$rep.json 2>/dev/null || { echo "lap $v failed"; exit 1; }
  show $D/lap_$v$rep.json lap_$v$rep
done
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/c3_b.json 2>/dev/null || { echo "c3 failed"; exit 1; }
show $D/c3_b.json c3_b
cp $L/libsgp_b.so $L/libsgp.so
B="python3 bench.py --mode fitc --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_b -o run -- $B > $D/pmc_b.json 2> $D/pmc_b.err || { tail -20 $D/pmc_b.err; exit 1; }
echo ok
