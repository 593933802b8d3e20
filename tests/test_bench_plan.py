"""bench.py's --gpus semantics (plan_run): N always means N GPUs, never a silent one-GPU run.

Under torch.distributed.run --gpus must equal WORLD_SIZE; without it, N > 1 runs the
in-library multi-device context over devices 0..N-1 (the path the R drop-in's sgp_R_ctx_create
takes); N above the visible device count is an error.  The N = 1 line is unchanged.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def vis(k):
    return lambda: k


def test_single_gpu_default():
    assert bench.plan_run(1, None, {}, vis(0)) == ("single", [0])
    assert bench.plan_run(1, None, {}, vis(8)) == ("single", [0])


def test_torchrun_world_must_match():
    env = {"RANK": "0", "WORLD_SIZE": "8", "LOCAL_RANK": "0"}
    assert bench.plan_run(8, None, env, vis(8)) == ("torchrun", 8)
    with pytest.raises(bench.PlanError, match="WORLD_SIZE=8"):
        bench.plan_run(1, None, env, vis(8))
    with pytest.raises(bench.PlanError, match="WORLD_SIZE=8"):
        bench.plan_run(4, None, env, vis(8))
    env1 = {"RANK": "0", "WORLD_SIZE": "1"}
    assert bench.plan_run(1, None, env1, vis(1)) == ("torchrun", 1)
    with pytest.raises(bench.PlanError):
        bench.plan_run(2, None, env1, vis(8))


def test_without_torchrun_n_gpus_is_the_library_context():
    assert bench.plan_run(8, None, {}, vis(8)) == ("library", list(range(8)))
    assert bench.plan_run(2, None, {}, vis(8)) == ("library", [0, 1])
    with pytest.raises(bench.PlanError, match="only 1 device"):
        bench.plan_run(8, None, {}, vis(1))
    with pytest.raises(bench.PlanError, match="only 0 device"):
        bench.plan_run(2, None, {}, vis(0))
    with pytest.raises(bench.PlanError, match="at least one"):
        bench.plan_run(0, None, {}, vis(8))
    with pytest.raises(bench.PlanError, match="without RANK"):
        bench.plan_run(2, None, {"WORLD_SIZE": "2"}, vis(8))


def test_devices_list():
    assert bench.plan_run(1, [0, 0, 0], {}, vis(1)) == ("library", [0, 0, 0])
    assert bench.plan_run(2, [0, 1, 0, 1], {}, vis(2)) == ("library", [0, 1, 0, 1])
    with pytest.raises(bench.PlanError, match="distinct"):
        bench.plan_run(4, [0, 1], {}, vis(8))
    with pytest.raises(bench.PlanError, match="visible"):
        bench.plan_run(1, [0, 3], {}, vis(2))
    with pytest.raises(bench.PlanError, match="not under torchrun"):
        bench.plan_run(1, [0], {"RANK": "0", "WORLD_SIZE": "1"}, vis(1))


def test_command_line_refuses_before_any_gpu_work():
    """The CLI exits non-zero (argparse error, status 2) on a mismatch, without touching a GPU
    (this container has none; a silent fallback would go on to build the problem)."""
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1",
                        "--no-cpu-baseline"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 2, r.stderr.decode()[-2000:]
    assert b"WORLD_SIZE=2" in r.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""   # no device here anyway
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                        "--no-cpu-baseline"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=300)
    assert r.returncode == 2, r.stderr.decode()[-2000:]
    assert b"device(s) are visible" in r.stderr
