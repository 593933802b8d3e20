#!/bin/bash
# Round-2 counter evidence on the GPU box (each PMC pass a run of its own, no trace domains):
#   store_bw micro (write-bandwidth ceiling of the builder's stream), kernel-trace stats of the
#   C3 bench, FETCH_SIZE / WRITE_SIZE passes, and two SQ passes (MFMA busy, VALU activity,
#   issue stalls) for k_build_knm_mfma, k_syrk_blk, k_contract and k_gj_step.
#   usage (inside gpurun): bash tools/gpu_pmc_r2.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
step() { echo "== $*"; }
step store_bw
timeout -k 10 120 ./tools/micro/store_bw > $D/store_bw.txt 2>&1 || { tail -5 $D/store_bw.txt; exit 1; }
cat $D/store_bw.txt
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/k.json 2> $D/k.err || { tail -20 $D/k.err; exit 1; }
step pmc-fetch
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pf -o run -- $B > $D/pf.json 2> $D/pf.err || { tail -20 $D/pf.err; exit 1; }
step pmc-write
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $D/pw -o run -- $B > $D/pw.json 2> $D/pw.err || { tail -20 $D/pw.err; exit 1; }
step pmc-sq1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/ps1 -o run -- $B > $D/ps1.json 2> $D/ps1.err || { tail -20 $D/ps1.err; exit 1; }
step pmc-sq2
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/ps2 -o run -- $B > $D/ps2.json 2> $D/ps2.err || { tail -20 $D/ps2.err; exit 1; }
ls -R $D | head -40
echo ok
