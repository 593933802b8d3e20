#!/bin/bash
# One SQ counter pass per library (product "cur" and tools/ab/<variant>) on one bench workload:
#   bash tools/pmc_ab.sh TAG "VARIANTS" BENCH_ARGS...
# -> gpurun_out/<TAG>_<variant>/ (csv); summarise with tools/pmc_summary.py.
set -o pipefail
T=$1; VARS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in cur $VARS; do
  if [ "$v" = cur ]; then unset SGP_AB_LIB; else export SGP_AB_LIB=tools/ab/$v/libsgp.so; fi
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_$v -o run -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$v.log 2>&1 || { echo "pmc $v failed"; tail -20 gpurun_out/${T}_$v.log; exit 1; }
  echo "pmc $v done"
done
