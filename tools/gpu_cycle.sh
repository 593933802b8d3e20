#!/bin/bash
# usage: gpu_cycle.sh TAG  -> tests + bench + pmc b pass into gpurun_out/TAG
T=$1
timeout 2400 /usr/local/graft/bin/gpurun --timeout 900 -- "mkdir -p gpurun_out/$T && export TMPDIR=/tmp && timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/$T/pytest.log 2>&1 && timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err && timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/b -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err; echo rc=\$?" 2>&1 | grep -v "^\[gpurun\] sending"
tail -2 gpurun_out/$T/pytest.log
python3 -c "
import json; r=json.load(open('gpurun_out/$T/bench.json')); print(r['value'], r['roofline']['achieved'], r['phases_ms'])"
python3 tools/pmc_summary.py gpurun_out/$T/b/run_counter_collection.csv | grep -v "SQ_\|GRBM"
