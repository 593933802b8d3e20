# round 5: persistent GJ with 16-byte sc1 loads, P_k kept across a workgroup's tasks, pipelined
# pivot sweeps, pivot blocks without a barrier -- micro, parity, A/B (gj8b: 8-byte loads, old pivot;
# nopipe: 16-byte loads, old pivot; nopiv2: 16-byte loads, pipelined sweeps, old block structure)
set -o pipefail
mkdir -p gpurun_out/gj16
timeout -k 10 60 ./tools/micro/gj_sweep > gpurun_out/gj16/sweep_micro.txt 2>&1 || { cat gpurun_out/gj16/sweep_micro.txt; exit 1; }
cat gpurun_out/gj16/sweep_micro.txt
timeout -k 10 150 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_gpu_vi.py > gpurun_out/gj16/t_vi.log 2>&1 || { tail -40 gpurun_out/gj16/t_vi.log; exit 1; }
tail -1 gpurun_out/gj16/t_vi.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_determinism.py tests/test_gpu_fitc.py \
  tests/test_gpu_laplace.py tests/test_gpu_multi.py tests/test_gpu_full.py tests/test_gpu_predict.py > gpurun_out/gj16/tests.log 2>&1 || { tail -40 gpurun_out/gj16/tests.log; exit 1; }
tail -1 gpurun_out/gj16/tests.log
bash tools/ab.sh gj16sh 2 "gj8b nopipe nopiv2" --config C3 --n 125000 --steps 40 --warmup 4 || exit 1
bash tools/ab.sh gj16c2 3 "gj8b nopipe nopiv2" --config C2 --steps 300 --warmup 20 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gj16/c2 -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gj16/c2k.json 2> gpurun_out/gj16/c2k.err || { tail -20 gpurun_out/gj16/c2k.err; exit 1; }
python3 tools/trace_eval.py gpurun_out/gj16/c2/run_kernel_trace.csv > gpurun_out/gj16/c2_timeline.txt && tail -3 gpurun_out/gj16/c2_timeline.txt
