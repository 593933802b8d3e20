"""bench.py's N > 1 control flow (the driver's scaling runs) on the one-GPU box.

`SGP_BENCH_REHEARSE=1` puts every rank on device 0 with gloo collectives, so the row sharding,
the barriers around the timed steps, the max-over-ranks timing and rank 0's single JSON line
run exactly as under `torch.distributed.run --nproc-per-node N` on an 8-GPU node (where the
collectives are RCCL).  The line is checked for the contract fields, and its objective for
agreement with a one-rank run of the same workload (the all-reduced partial sums must give the
same ELBO to rounding).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = 20000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(nproc, extra_env, mode):
    env = dict(os.environ, **extra_env)
    args = ["bench.py", "--gpus", str(nproc), "--steps", "2", "--warmup", "1",
            "--no-cpu-baseline", "--rows", str(ROWS), "--mode", mode]
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]   # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("mode", ["vi", "fitc", "laplace"])
def test_two_rank_bench_line_matches_one_rank(mode):
    one = _bench(1, {}, mode)
    two = _bench(2, {"SGP_BENCH_REHEARSE": "1"}, mode)
    assert two["n_gpus"] == 2 and two["steps"] == 2 and two["warmup"] == 1
    assert two["config"]["parallelism"] == "rows2" and two["config"]["n"] == ROWS
    assert two["value"] > 0 and two["ms_per_step"] > 0
    assert abs(two["value"] * two["ms_per_step"] - 1e3) < 1e-6 * 1e3   # evals/s of the whole job
    assert abs(two["objective"] - one["objective"]) <= 1e-9 * abs(one["objective"])
