#!/bin/bash
# One parametrised launcher for the GPU box (replaces round 5's one-off tools/gpu_r5_*.sh; they
# are in git history).  Every step runs under its own time limit; the first failing step ends
# the call (no retries).  Results go under gpurun_out/$OUT (default gpurun_out/run).
#   usage (inside gpurun): bash tools/gpu_run.sh STEP [STEP ...]
#   steps:
#     suite[:PATTERN]   pytest -m gpu (PATTERN: a -k expression), log in $D/suite.log
#     tests:FILES       pytest -m gpu on the comma-separated test files only
#     bench             the default bench line (bench.py, cpu_baseline included) -> $D/bench.json
#     prof              rocprofv3 --kernel-trace --stats of the bench command -> $D/k/
#     modes             the secondary lines: C2, the n = 125 000 shard, FITC, C5, knots, the
#                       in-library 8-shard composition -> $D/run_*.json
#     c2x4              four C2 lines in a row (the C2 measure) -> $D/c2_*.json
#     c2trace           rocprofv3 --kernel-trace --stats of a C2 line and the timeline of its last
#                       evaluation (tools/trace_eval.py) -> $D/c2k/, $D/c2_timeline.txt
#     pmc               WRITE_SIZE / FETCH_SIZE passes of the bench command (one counter set
#                       per run, kernel trace only) -> $D/pmc_*/
#     builderpmc        counter passes over tools/builder_probe.py (K12 builder + store ceiling)
#     ab:TAG:REPS:VARS:ARGS   tools/ab.sh TAG REPS "VARS" ARGS (ARGS with '+' for spaces)
set -o pipefail
D=gpurun_out/${OUT:-run}
mkdir -p "$D"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp

last_json() {   # the last JSON line of a file, as a one-line summary
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['value'],3), round(d['ms_per_step'],4), d.get('roofline',{}).get('frac'), [ (k['kernel'][:10], round(k['frac'],3), round(k.get('frac_of_store_ceiling',0),3)) for k in d.get('kernel_rooflines',[])])" "$1" "$2"
}

for step in "$@"; do
  case "$step" in
    suite*)
      pat=${step#suite}; pat=${pat#:}
      timeout -k 10 1500 python -u -m pytest --maxfail=5 -v -s --timeout 300 --timeout-method thread \
        -m gpu ${pat:+-k "$pat"} tests/ > "$D/suite.log" 2>&1 || { tail -40 "$D/suite.log"; exit 1; }
      tail -1 "$D/suite.log" ;;
    tests:*)
      files=$(echo "${step#tests:}" | tr ',' ' ')
      timeout -k 10 1200 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
        $files > "$D/tests.log" 2>&1 || { tail -60 "$D/tests.log"; exit 1; }
      tail -1 "$D/tests.log" ;;
    bench)
      timeout -k 10 500 python3 bench.py > "$D/bench.json" 2> "$D/bench.err" || { tail -20 "$D/bench.err"; exit 1; }
      last_json "$D/bench.json" bench ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/k" -o run -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$D/k.json" 2> "$D/k.err" || { tail -20 "$D/k.err"; exit 1; }
      last_json "$D/k.json" prof ;;
    modes)
      for a in "--config C2 --steps 300 --warmup 20" "--n 125000 --steps 40 --warmup 4" \
               "--mode fitc --steps 6 --warmup 2" "--config C5 --mode laplace --steps 10 --warmup 2" \
               "--knots --steps 6 --warmup 2" "--devices 0,0,0,0,0,0,0,0 --steps 6 --warmup 2"; do
        f="$D/run_$(echo $a | tr -c 'a-zA-Z0-9' '_').json"
        timeout -k 10 300 python3 bench.py --no-cpu-baseline $a > "$f" 2> "$D/run.err" || { tail -20 "$D/run.err"; exit 1; }
        last_json "$f" "$a"
      done ;;
    c2x4)
      for r in 1 2 3 4; do
        timeout -k 10 200 python3 bench.py --no-cpu-baseline --config C2 --steps 300 --warmup 20 \
          > "$D/c2_$r.json" 2> "$D/run.err" || { tail -20 "$D/run.err"; exit 1; }
        last_json "$D/c2_$r.json" "c2 $r"
      done ;;
    c2trace)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/c2k" -o run -- \
        python3 bench.py --no-cpu-baseline --config C2 --steps 60 --warmup 5 > "$D/c2k.json" 2> "$D/c2k.err" || { tail -20 "$D/c2k.err"; exit 1; }
      python3 tools/trace_eval.py "$D/c2k/run_kernel_trace.csv" "k_contract<8, 0, false, false, false" > "$D/c2_timeline.txt" && tail -1 "$D/c2_timeline.txt" ;;
    pmc)
      for ctr in "FETCH_SIZE" "WRITE_SIZE"; do
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$D/pmc_$ctr" -o run -- \
          python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$D/pmc_$ctr.json" 2> "$D/pmc_$ctr.err" || { tail -20 "$D/pmc_$ctr.err"; exit 1; }
        echo "pmc $ctr done"
      done ;;
    builderpmc)
      # the K12 builder and the store ceiling kernel in one process, one counter set per run
      i=0
      for set in "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum" "TCC_EA0_WRREQ_STALL_sum" \
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$D/bpmc_$i" -o run -- \
          python3 tools/builder_probe.py > "$D/bpmc_$i.log" 2>&1 || { tail -20 "$D/bpmc_$i.log"; exit 1; }
        tail -1 "$D/bpmc_$i.log"
      done ;;
    ab:*)
      IFS=: read -r _ tag reps vars args <<< "$step"
      bash tools/ab.sh "$tag" "$reps" "$vars" $(echo "$args" | tr '+' ' ') || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
