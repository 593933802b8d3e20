#!/bin/bash
# C2: parity of the VI path, the bench line, the host-issue profile and a HIP API + kernel
# trace (tools/api_gap.py).  usage (inside gpurun): bash tools/gpu_r3_api.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_edges.py tests/test_gpu_knots.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 200 python3 bench.py --config C2 --steps 40 --warmup 3 --no-cpu-baseline > $D/c2.json 2>/dev/null || { echo "c2 failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c2.json').read().strip().splitlines()[-1]); print('c2', round(d['value'],1), round(d['ms_per_step'],4), d['phases_ms'])"
timeout -k 10 120 python3 tools/host_overhead.py C2 - 60 > $D/host_c2.txt 2>&1 || { echo "host failed"; exit 1; }
cat $D/host_c2.txt
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $D/c2a -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/c2a.json 2> $D/c2a.err || { tail -20 $D/c2a.err; exit 1; }
python3 tools/api_gap.py $D/c2a > $D/c2_api_gap.txt 2>&1 || true
echo ok
