"""Regression test of the two-RCCL-copies fault (multi.hip's `Rccl` binding, round 5).

A process that runs libsgp's in-library multi-device context AND torch.distributed holds two
RCCL users.  When libsgp linked ROCm's librccl.so.1 at load time and was loaded before torch,
the process carried two RCCL copies with interposed symbols, and their exit-time destructors
freed the same objects ("double free or corruption" at exit).  libsgp now opens RCCL with
dlopen at the first multi-device context (an RCCL already in the process is reused, otherwise
ROCm's is opened RTLD_LOCAL).  The order that used to fail: libsgp loaded and a multi context
created (and evaluated) BEFORE torch initialises its own RCCL, then torch's all-reduce, then a
normal exit.  The child must exit 0 with no allocator abort in its output.
"""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {root!r})
    import numpy as np
    import sparsergps_amd as S
    from sparsergps_amd.workloads import make_gaussian_problem
    assert "torch" not in sys.modules
    P = make_gaussian_problem("C2", n=3000, m=64)
    th = np.array(list(P["cov_par"].values()))
    ctx = S.SparseGPContext(P["X"], P["y"], P["mu"], m_max=64, devices=[0, 0])
    o, g = ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
    print("LIBSGP_FIRST", o, flush=True)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    t = torch.ones(1024, dtype=torch.float64, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print("TORCH_ALLREDUCE", float(t[0]), flush=True)
    o2, g2 = ctx.eval_vi(th, "sqexp", P["U"], P["delta"])
    assert o2 == o and np.array_equal(g2, g)
    ctx.close()
    dist.destroy_process_group()
    print("EXITING", flush=True)
""")


def test_libsgp_rccl_before_torch_rccl_exits_cleanly():
    from sparsergps_amd import _lib
    _lib.require_gpu()
    port = 29500 + (os.getpid() % 1000)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, port=port)], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=110)
    out = r.stdout.decode(errors="replace")
    print(out[-3000:])
    assert r.returncode == 0, out[-4000:]
    for s in ("LIBSGP_FIRST", "TORCH_ALLREDUCE 1.0", "EXITING"):
        assert s in out, out[-3000:]
    for bad in ("double free", "corruption", "free(): invalid", "Aborted", "Segmentation"):
        assert bad not in out, out[-4000:]
