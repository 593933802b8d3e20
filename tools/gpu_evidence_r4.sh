#!/bin/bash
# Round-4 evidence pass on the GPU box: GPU tests, the default bench line (with the CPU
# baseline), its rocprofv3 kernel-trace summary, separate PMC passes (FETCH_SIZE, WRITE_SIZE,
# two SQ sets, L2 hit/miss), the secondary modes, the 8-GPU shard-size line
# and the torchrun N=1 (RCCL) rehearsal.
#   usage (inside gpurun): bash tools/gpu_evidence_r4.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
step() { echo "== $* $(date +%T)"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=5 --timeout 420 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
step bench
timeout -k 10 400 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cut -c1-300 $D/bench.json
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
step pmc-l2
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $D/pl2 -o run -- $B > $D/pl2.json 2> $D/pl2.err || echo "L2 pass failed (continuing)"
step modes
timeout -k 10 300 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc.json 2> $D/fitc.err || exit 1
timeout -k 10 300 python3 bench.py --mode laplace --steps 10 --warmup 2 --no-cpu-baseline > $D/laplace.json 2> $D/laplace.err || exit 1
timeout -k 10 300 python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || exit 1
timeout -k 10 300 python3 bench.py --knots --no-cpu-baseline > $D/knots.json 2> $D/knots.err || exit 1
step c2-trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2k -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2k.json 2> $D/c2k.err || { tail -20 $D/c2k.err; exit 1; }
step shards
for nn in 125000; do
  timeout -k 10 200 python3 bench.py --rows $nn --steps 10 --warmup 3 --no-cpu-baseline > $D/rows$nn.json 2> $D/rows$nn.err || exit 1
done
step torchrun
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --rows 125000 --steps 10 --warmup 3 --no-cpu-baseline > $D/trun.json 2> $D/trun.err || { tail -20 $D/trun.err; exit 1; }
python3 - "$D" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split("/")[-1], round(d["value"], 3), round(d["ms_per_step"], 3))
    except Exception:
        pass
PY
echo "pytest rc=$rc"
