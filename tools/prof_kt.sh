#!/bin/bash
# Kernel traces of the product library ("cur") and variant libraries (tools/ab/<name>) on one
# bench workload: bash tools/prof_kt.sh TAG "VARIANTS" BENCH_ARGS...
# Writes gpurun_out/<TAG>_<variant>/run_results.db; summarise with tools/kt_summary.py.
set -o pipefail
T=$1; VARS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in cur $VARS; do
  if [ "$v" = cur ]; then unset SGP_AB_LIB; else export SGP_AB_LIB=tools/ab/$v/libsgp.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_$v -o run -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$v.log 2>&1 || { echo "trace $v failed"; tail -20 gpurun_out/${T}_$v.log; exit 1; }
  echo "traced $v"
done
