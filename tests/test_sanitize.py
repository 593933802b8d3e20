"""ASan + UBSan build of libsgp's host code, driven through its C ABI without a GPU.

SURVEY.md sec. 5 ("race detection / sanitizers"): every csrc/*.hip translation unit is
compiled with -fsanitize=address,undefined on the host side only (each -fsanitize= behind
-Xarch_host: GPU sanitizers are not available for gfx950 on this pool and the device code is
never executed here), linked with tests/sanitize/host_driver.c, and run.  The driver covers
the host-only entry points (per-pair kernels, reduction-size queries) and the argument checks
of every entry point; any sanitizer report aborts the run (halt_on_error, no recovery).
Objects go to build/asan/ (git-ignored); the build takes ~1 minute on 8 cores.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sparsergps_amd", "csrc")
OUT = os.path.join(ROOT, "build", "asan")
from sparsergps_amd._build import SOURCES  # noqa: E402  (every translation unit)
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    pytest.skip("hipcc not available")


def test_host_abi_under_asan_ubsan():
    cc = _hipcc()
    os.makedirs(OUT, exist_ok=True)
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(OUT, src.replace(".hip", ".o"))
        objs.append(obj)
        cmd = [cc, "-O1", "-g", "--offload-arch=gfx950", "-std=c++17", "-fPIC", *SAN,
               "-Wno-unused-result", "-c", os.path.join(CSRC, src), "-o", obj]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate()
        assert p.returncode == 0, out.decode(errors="replace")[-4000:]
    exe = os.path.join(OUT, "host_driver")
    drv = os.path.join(ROOT, "tests", "sanitize", "host_driver.c")
    res = subprocess.run([cc, "-O1", "-g", "-x", "c++", *SAN, "-I", os.path.join(ROOT, "include"),
                          drv, "-x", "none", *objs, "--offload-arch=gfx950",
                          "-fsanitize=address,undefined", "-ldl", "-lpthread", "-o", exe],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    assert res.returncode == 0, res.stdout.decode(errors="replace")[-4000:]
    env = dict(os.environ)
    # leaks inside the HIP runtime's own initialisation are not this library's; every other
    # ASan / UBSan report aborts the driver
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    run = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env,
                         timeout=300)
    text = run.stdout.decode(errors="replace")
    assert run.returncode == 0, text[-6000:]
    assert "all checks passed" in text
    assert "runtime error" not in text and "AddressSanitizer" not in text, text[-6000:]
