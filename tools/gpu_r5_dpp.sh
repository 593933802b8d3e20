# round 5: the pivot sweeps with one DPP64 fmac per register -- parity, A/B against r5h4
set -o pipefail
D=gpurun_out/dpp
mkdir -p $D
timeout -k 10 150 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_vi.py > $D/t_vi.log 2>&1 || { tail -40 $D/t_vi.log; exit 1; }
tail -1 $D/t_vi.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_fitc.py \
  tests/test_gpu_laplace.py tests/test_gpu_multi.py tests/test_gpu_full.py tests/test_gpu_predict.py tests/test_gpu_rccl.py > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
bash tools/ab.sh dpc2 3 "r5h4" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh dpsh 3 "r5h4" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
bash tools/ab.sh dpc3 2 "r5h4" --steps 10 --warmup 2 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2k.json 2> $D/c2k.err || { tail -20 $D/c2k.err; exit 1; }
python3 tools/trace_eval.py $D/c2/run_kernel_trace.csv "k_contract<8, 0, false, false, false" > $D/c2_timeline.txt && tail -3 $D/c2_timeline.txt
