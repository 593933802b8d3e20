"""Build libsgp.so (hipcc, gfx950) in-tree.

The shared library lands in sparsergps_amd/lib/libsgp.so so it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libsgp.so")
SOURCES = ["capi.hip", "k_cov.hip", "k_mfma.hip", "k_dense.hip", "k_lap.hip"]
HEADERS = ["sgp_internal.h", os.path.join("..", "..", "include", "sgp.h")]
ARCH = os.environ.get("SGP_OFFLOAD_ARCH", "gfx950")


class HipccMissing(RuntimeError):
    """No hipcc on this machine (the only case in which an existing library may be reused)."""


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise HipccMissing("hipcc not found: cannot build libsgp.so")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


# Per-source compiler flags.  k_dense.hip: MFMA accumulators in VGPRs -- the Gauss-Jordan
# pivot's scalar sweeps read and rewrite its accumulator tiles between MFMA blocks, and in AGPRs
# every sweep paid v_accvgpr_read / write moves (pivot 10.8-11.3 -> 10.2-10.6 us, one m = 1024
# chain 356-359 -> 342-345 us: profiles/r3/gj_vgpr_form_ab.txt)
FILE_FLAGS = {"k_dense.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every HIP source for gfx950 into lib/libsgp.so (incremental per object)."""
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    cc = hipcc()
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(LIBDIR, src.replace(".hip", ".o"))
        objs.append(obj)
        # SGP_HIPCC_DEFS: extra -D flags for A/B experiment builds (tools/ab_*.sh), never set
        # for the product library
        extra = os.environ.get("SGP_HIPCC_DEFS", "").split()
        cmd = [cc, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result",
               *FILE_FLAGS.get(src, []), *extra, "-c", os.path.join(CSRC, src), "-o", obj]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed ({' '.join(cmd)}):\n{out.decode(errors='replace')}")
        if verbose and out:
            print(out.decode(errors="replace"))
    tmp = LIB + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stdout.decode(errors='replace')}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
