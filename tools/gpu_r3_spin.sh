#!/bin/bash
# Round 3: host spin-wait on the readback's pinned sequence word (SGP_SPIN_WAIT=1) against
# hipStreamSynchronize (0): VI / Laplace parity with the spin, C2 A/B and the host-issue profile.
#   usage (inside gpurun): bash tools/gpu_r3_spin.sh TAG
set -o pipefail
T=$1
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
SGP_SPIN_WAIT=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_vi.py tests/test_gpu_laplace.py tests/test_gpu_fitc.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for rep in 1 2 3; do
for v in 0 1; do
  SGP_SPIN_WAIT=$v timeout -k 10 200 python3 bench.py --config C2 --steps 60 --warmup 5 --no-cpu-baseline > $D/c2_$v$rep.json 2>/dev/null || { echo "c2 $v failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/c2_$v$rep.json').read().strip().splitlines()[-1]); print('spin$v rep$rep', round(d['value'],1), round(d['ms_per_step'],4))"
done
done
SGP_SPIN_WAIT=1 timeout -k 10 120 python3 tools/host_overhead.py C2 - 60 > $D/host_c2_spin.txt 2>&1 || { echo "host failed"; exit 1; }
SGP_SPIN_WAIT=0 timeout -k 10 120 python3 tools/host_overhead.py C2 - 60 > $D/host_c2_sync.txt 2>&1 || { echo "host failed"; exit 1; }
grep -v amdgpu.ids $D/host_c2_spin.txt $D/host_c2_sync.txt
echo ok
