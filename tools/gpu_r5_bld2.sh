# round 5: where VI's builder time goes -- kernel trace of VI and FITC at C3, and VI's builder without t
set -o pipefail
mkdir -p gpurun_out/bld2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bld2/vi -o vi -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/bld2/vi.json 2>gpurun_out/bld2/vi.err || { tail gpurun_out/bld2/vi.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bld2/fitc -o fitc -- python3 bench.py --no-cpu-baseline --mode fitc --steps 4 --warmup 2 > gpurun_out/bld2/fitc.json 2>gpurun_out/bld2/fitc.err || { tail gpurun_out/bld2/fitc.err; exit 1; }
bash tools/ab.sh bld2 2 "vinot" --steps 10 --warmup 2 || exit 1
