#!/bin/bash
# RCCL all-reduce time of the C4 exchange buffers at world size 1, the torchrun N = 1 shard line
# (collectives on), and the LDS-conflict counters of the m x m kernels after the odd-stride fix.
#   usage (inside gpurun): bash tools/gpu_r3_misc.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 180 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 tools/rccl_allreduce_time.py > $D/rccl.json 2> $D/rccl.err || { echo "rccl failed"; tail -20 $D/rccl.err; exit 1; }
cat $D/rccl.json
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --rows 125000 --steps 20 --warmup 3 --no-cpu-baseline > $D/trun125.json 2> $D/trun125.err || { echo "torchrun bench failed"; tail -20 $D/trun125.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/trun125.json').read().strip().splitlines()[-1]); print('trun125', round(d['value'],2), round(d['ms_per_step'],3), d.get('collectives'), d['phases_ms'])"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/pl -o run -- $B > $D/pl.json 2> $D/pl.err || { tail -20 $D/pl.err; exit 1; }
python3 tools/pmc_summary.py $D/pl/run_counter_collection.csv k_gj_step k_gemm64 "k_contract<8, 0" k_syrk_blk
echo ok
