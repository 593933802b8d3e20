#!/bin/bash
# Round 3: rocprofv3 kernel statistics of the secondary configurations (C2, FITC at C3, Laplace
# at C5) and one SQ counter pass each for FITC and Laplace.  usage: bash tools/gpu_r3_modes.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2.json 2> $D/c2.err || { tail -20 $D/c2.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/fitc -o run -- python3 bench.py --mode fitc --steps 3 --warmup 1 --no-cpu-baseline > $D/fitc.json 2> $D/fitc.err || { tail -20 $D/fitc.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/lap -o run -- python3 bench.py --mode laplace --steps 5 --warmup 2 --no-cpu-baseline > $D/lap.json 2> $D/lap.err || { tail -20 $D/lap.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_fitc -o run -- python3 bench.py --mode fitc --steps 2 --warmup 1 --no-cpu-baseline > $D/pmc_fitc.json 2> $D/pmc_fitc.err || { tail -20 $D/pmc_fitc.err; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/pmc_lap -o run -- python3 bench.py --mode laplace --steps 3 --warmup 1 --no-cpu-baseline > $D/pmc_lap.json 2> $D/pmc_lap.err || { tail -20 $D/pmc_lap.err; exit 1; }
echo ok
