#!/bin/bash
# Summarise a tools/gpu_check.sh run (here, after gpurun merged gpurun_out/).
T=$1
tail -1 gpurun_out/$T/pytest.log
python3 -c "
import json; r=json.load(open('gpurun_out/$T/bench.json')); print(round(r['value'],3), 'evals/s', round(r['ms_per_step'],3), 'ms', 'con', round(r['roofline']['achieved'],2), 'TF'); print(r['phases_ms'])"
python3 tools/trace_eval.py gpurun_out/$T/k/run_kernel_trace.csv > gpurun_out/$T/timeline.txt && tail -1 gpurun_out/$T/timeline.txt
