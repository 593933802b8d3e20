#!/bin/bash
# FITC weighted SYRK with t: parity tests, the C3 FITC bench line (phase times) and two SQ
# counter passes over a short FITC run.  usage (inside gpurun): bash tools/gpu_r3_fitc.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fitc.py tests/test_gpu_laplace.py tests/test_gpu_configs.py tests/test_gpu_vi.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python3 bench.py --mode fitc --no-cpu-baseline > $D/fitc.json 2> $D/fitc.err || { echo "bench failed"; tail -20 $D/fitc.err; exit 1; }
timeout -k 10 300 python3 bench.py --mode laplace --no-cpu-baseline > $D/lap.json 2> $D/lap.err || { echo "bench failed"; tail -20 $D/lap.err; exit 1; }
B="python3 bench.py --mode fitc --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/ps1 -o run -- $B > $D/ps1.json 2> $D/ps1.err || { tail -20 $D/ps1.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/ps2 -o run -- $B > $D/ps2.json 2> $D/ps2.err || { tail -20 $D/ps2.err; exit 1; }
python3 - "$D" <<'PY'
import json, sys
for f in ("fitc", "lap"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"], 3), round(d["ms_per_step"], 3), d["phases_ms"])
PY
echo ok
