"""The multi-device context's host orchestration at G > 1 device groups, without a GPU.

multi.hip's worker pool, barriers with votes and job bodies live in
sparsergps_amd/csrc/sgp_pool.h (HIP- and RCCL-free); tests/pool/pool_driver.cc drives them with
G = 1, 2, 3 and 8 fake device groups (one or two shards each) whose all-reduce only enqueues and
whose next phase waits for it with a deadline (a hang is reported, not suffered).  Cases: clean
VI / FITC and Laplace evaluations against serially computed sums (every group the same), a
failure injected in one group at every phase before, between and after the collectives, one
group's collective failing to enqueue after its peers' were queued (the post-collective vote),
a Laplace step failure and a disagreeing NR stop vote (R/newtrap_sparseGP.R:77-150 -- every
group must stop at the same step).  Every faulted run must end every worker with the failing
group's status (peers ABORTED), leave no group waiting, and the next clean evaluation must be
right again.  Built twice: under ThreadSanitizer (halt on the first report) and optimised with
more repetitions.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "tests", "pool", "pool_driver.cc")
OUT = os.path.join(ROOT, "build", "pool")


def _gxx():
    c = shutil.which("g++")
    if not c:
        pytest.skip("g++ not available")
    return c


def _build(name, flags):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    res = subprocess.run([_gxx(), "-std=c++17", "-g", "-pthread", "-Wall", "-Wextra", "-Werror",
                          *flags, DRV, "-o", exe], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT)
    assert res.returncode == 0, res.stdout.decode(errors="replace")[-4000:]
    return exe


def _run(exe, reps, env=None):
    run = subprocess.run([exe, str(reps)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         timeout=600, env=env)
    text = run.stdout.decode(errors="replace")
    assert run.returncode == 0, text[-6000:]
    assert "cases passed" in text, text[-2000:]
    return text


def test_orchestration_under_tsan():
    exe = _build("pool_tsan", ["-O1", "-fsanitize=thread"])
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1:second_deadlock_stack=1"
    text = _run(exe, 3, env)
    assert "ThreadSanitizer" not in text, text[-6000:]


def test_orchestration_many_interleavings():
    exe = _build("pool_opt", ["-O2"])
    _run(exe, 20)
