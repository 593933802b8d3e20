"""The RCCL product path on hardware: torch.distributed "nccl" (= RCCL over xGMI) at world size
1 with the collectives forced on (sparsergps_amd/dist.py force_collectives), so every
all-reduce of the row-sharded VI / FITC / Laplace evaluations runs through RCCL on the
library's stream exactly as on an 8-GPU node.  Includes the C4 shard shape (n = 125 000,
m = 1024, d = 8) checked against the row-chunked adjoint model (oracle/adjoint_chunked.py).

The worker (tests/rccl_worker.py) is a fresh child process: the process group must be created
before anything else touches the GPU, which the pytest process already has.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_rccl_world_size_one_forced_collectives():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_worker.py")], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=400)
    out = res.stdout.decode(errors="replace")
    print(out)
    cases = [json.loads(line) for line in out.splitlines() if line.startswith("{")]
    names = {c["case"] for c in cases}
    assert {"vi_rccl", "fitc_rccl", "laplace_rccl", "knots_rccl",
            "c4_shard_125000_rccl"} <= names, out[-3000:]
    for c in cases:
        assert c["ok"], c
    assert res.returncode == 0, out[-3000:]
