#!/bin/bash
# Round 3: branch-free t slice in the with-t SYRK.  Parity (b = new library), FITC A/B against
# the previous library (a), the Laplace line, the VERDICT's PMC pass over the weighted SYRK,
# and the contraction probe at C2 / C3 shapes.  usage (inside gpurun): bash tools/gpu_r3_c.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
L=sparsergps_amd/lib
cp $L/libsgp_b.so $L/libsgp.so
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_configs.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2; do
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -k 10 200 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc_$v$rep.json 2>/dev/null || { echo "fitc $v failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$D/fitc_$v$rep.json').read().strip().splitlines()[-1]); print('$v$rep', round(d['value'],3), d['phases_ms']['syrk'], d['phases_ms']['syrk_omega'])"
done
done
cp $L/libsgp_b.so $L/libsgp.so
timeout -k 10 200 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap.json 2>/dev/null || { echo "lap failed"; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$D/lap.json').read().strip().splitlines()[-1]); print('lap', round(d['value'],3), d['phases_ms'])"
B="python3 bench.py --mode fitc --steps 2 --warmup 1 --no-cpu-baseline"
for v in a b; do
  cp $L/libsgp_$v.so $L/libsgp.so
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_$v -o run -- $B > $D/pmc_$v.json 2> $D/pmc_$v.err || { tail -20 $D/pmc_$v.err; exit 1; }
done
cp $L/libsgp_b.so $L/libsgp.so
cd tools/micro
timeout -k 10 60 ./con_trace ../../$D/con_c2.csv 100000 256 > ../../$D/con_c2.txt && timeout -k 10 60 ./con_trace ../../$D/con_c3.csv 131072 1024 > ../../$D/con_c3.txt || { echo "con_trace failed"; exit 1; }
cat ../../$D/con_c2.txt ../../$D/con_c3.txt
echo ok
