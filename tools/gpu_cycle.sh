#!/bin/bash
# Developer loop on the GPU box: GPU tests, one bench line, then either a PMC pass (default)
# or a kernel trace (MODE=kt).  Results land in gpurun_out/TAG.
#   usage: tools/gpu_cycle.sh TAG [pmc|kt]
T=$1
MODE=${2:-pmc}
if [ "$MODE" = kt ]; then
  PROF="rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/k -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$T/k.json 2> gpurun_out/$T/k.err"
else
  PROF="rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/b -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err"
fi
timeout 2400 /usr/local/graft/bin/gpurun --timeout 900 -- "mkdir -p gpurun_out/$T && export TMPDIR=/tmp && timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/$T/pytest.log 2>&1 && timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err && timeout -k 10 300 $PROF; echo rc=\$?" 2>&1 | grep -v "^\[gpurun\] sending"
tail -2 gpurun_out/$T/pytest.log
python3 -c "
import json; r=json.load(open('gpurun_out/$T/bench.json')); print(r['value'], r['roofline']['achieved'], r['phases_ms'])"
if [ "$MODE" = kt ]; then
  python3 tools/trace_eval.py gpurun_out/$T/k/run_kernel_trace.csv | tail -1
else
  python3 tools/pmc_summary.py gpurun_out/$T/b/run_counter_collection.csv | grep -v "SQ_\|GRBM"
fi
