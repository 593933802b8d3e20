"""Build libsgp.so (hipcc, gfx950) in-tree.

The shared library lands in sparsergps_amd/lib/libsgp.so so it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).

The product build takes no flags from the environment: experiment variants (-D knobs of
sgp_probe.h) are built by `build_variant()` into their own directory under tools/ab/, never
into lib/.  Every object records the compile flags it was built with in a stamp file beside
it (`<obj>.cmd`); an object is rebuilt when a source or header is newer than it or when its
flags differ from the stamp, so a library built with other flags can never be kept as the
product by an mtime check.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libsgp.so")
VARIANT_ROOT = os.path.join(ROOT, "tools", "ab")
SOURCES = ["capi.hip", "k_cov.hip", "k_mfma.hip", "k_dense.hip", "k_lap.hip", "multi.hip"]
HEADERS = ["sgp_internal.h", "sgp_probe.h", "sgp_multi.h", "sgp_pool.h",
           os.path.join("..", "..", "include", "sgp.h"),
           os.path.join("..", "..", "include", "sgp_diag.h")]
ARCH = "gfx950"


class HipccMissing(RuntimeError):
    """No hipcc on this machine (the only case in which an existing library may be reused)."""


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise HipccMissing("hipcc not found: cannot build libsgp.so")


# Per-source compiler flags.  k_dense.hip: MFMA accumulators in VGPRs -- the Gauss-Jordan
# pivot's scalar sweeps read and rewrite its accumulator tiles between MFMA blocks, and in AGPRs
# every sweep paid v_accvgpr_read / write moves (pivot 10.8-11.3 -> 10.2-10.6 us, one m = 1024
# chain 356-359 -> 342-345 us: profiles/r3/gj_vgpr_form_ab.txt)
FILE_FLAGS = {"k_dense.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _compile_flags(src, defs=()):
    return ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result",
            *FILE_FLAGS.get(src, []), *defs]


def _compile_cmd(cc, src, obj, defs=(), csrc=CSRC):
    return [cc, *_compile_flags(src, defs), "-c", os.path.join(csrc, src), "-o", obj]


# libdl: librccl is opened by the first sgp_ctx_create_multi context (multi.hip: reusing an
# RCCL the process already has, e.g. torch's; not a load-time dependency)
LINK_FLAGS = [f"--offload-arch={ARCH}", "-shared", "-fPIC", "-ldl", "-lpthread"]


def _link_cmd(cc, objs, out):
    return [cc, *LINK_FLAGS, "-o", out] + list(objs)


# The stamps hold the flags and inputs by name only (no compiler or repository path), so a
# snapshot of the tree that lands at another path (the GPU box) sees its objects as current.
def _stamp(path):
    return path + ".cmd"


def _read_stamp(path):
    try:
        with open(_stamp(path)) as f:
            return f.read()
    except OSError:
        return None


def _write_stamp(path, key):
    with open(_stamp(path), "w") as f:
        f.write(key)


def _obj_key(src, defs):
    return "\0".join([src, *_compile_flags(src, defs)])


def _lib_key(objs):
    return "\0".join([*LINK_FLAGS, *(os.path.basename(o) for o in objs)])


def _obj_stale(obj, key, src, csrc=CSRC):
    if not os.path.exists(obj) or _read_stamp(obj) != key:
        return True
    # a source depends on its own text and on every header (all sources include sgp_internal.h)
    t = os.path.getmtime(obj)
    deps = [os.path.join(csrc, src)] + [os.path.join(csrc, h) for h in HEADERS]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def _sources(csrc=CSRC):
    # an A/B build of an older revision compiles the translation units that revision has
    return [s for s in SOURCES if csrc == CSRC or os.path.exists(os.path.join(csrc, s))]


def _plan(outdir, defs, csrc=CSRC):
    objs, todo = [], []
    for src in _sources(csrc):
        obj = os.path.join(outdir, src.replace(".hip", ".o"))
        objs.append(obj)
        if _obj_stale(obj, _obj_key(src, defs), src, csrc):
            todo.append((src, obj))
    return objs, todo


def _lib_stale(lib, objs):
    if not os.path.exists(lib) or _read_stamp(lib) != _lib_key(objs):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(o) > t for o in objs)


def _build_into(outdir, lib, defs, force, verbose, csrc=CSRC):
    cc = hipcc()
    os.makedirs(outdir, exist_ok=True)
    objs, todo = _plan(outdir, defs, csrc)
    if force:
        todo = list(zip(_sources(csrc), objs))
    procs = []
    for src, obj in todo:
        cmd = _compile_cmd(cc, src, obj, defs, csrc)
        procs.append((src, cmd, obj,
                      subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = None
    for src, cmd, obj, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed = failed or f"hipcc failed ({' '.join(cmd)}):\n{out.decode(errors='replace')}"
            continue
        _write_stamp(obj, _obj_key(src, defs))
        if verbose and out:
            print(out.decode(errors="replace"))
    if failed:
        raise RuntimeError(failed)
    if not force and not todo and not _lib_stale(lib, objs):
        return lib
    tmp = lib + ".tmp"
    res = subprocess.run(_link_cmd(cc, objs, tmp), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stdout.decode(errors='replace')}")
    os.replace(tmp, lib)
    _write_stamp(lib, _lib_key(objs))
    return lib


def stale() -> bool:
    """True when build() would compile or link anything."""
    objs, todo = _plan(LIBDIR, ())
    return bool(todo) or _lib_stale(LIB, objs)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the HIP sources for gfx950 into lib/libsgp.so, recompiling only the objects
    whose source, headers or compile command changed."""
    if os.environ.get("SGP_HIPCC_DEFS"):
        raise RuntimeError("SGP_HIPCC_DEFS is not honoured by the product build; "
                           "use sparsergps_amd._build.build_variant() for A/B libraries")
    return _build_into(LIBDIR, LIB, (), force, verbose)


def build_variant(name: str, defs=(), force: bool = False, verbose: bool = False,
                  rev: str | None = None) -> str:
    """An experiment library in tools/ab/<name>/: extra -D flags (SGP_PROBE_BUILD implied)
    and/or the HIP sources of git revision `rev` (A/B against an earlier kernel).

    Load it with SGP_AB_LIB=<returned path> (sparsergps_amd._lib accepts only paths under
    tools/ab/).  The product lib/libsgp.so is never touched."""
    if not name or "/" in name or name.startswith("."):
        raise ValueError(f"bad variant name {name!r}")
    defs = ["-DSGP_PROBE_BUILD", *defs]
    outdir = os.path.join(VARIANT_ROOT, name)
    csrc = CSRC
    if rev is not None:
        # the revision's sources (csrc + include/sgp.h) exported under tools/ab/<name>/src
        src_root = os.path.join(outdir, "src")
        os.makedirs(src_root, exist_ok=True)
        for path in ["sparsergps_amd/csrc/" + f for f in SOURCES + HEADERS[:4]] + ["include/sgp.h", "include/sgp_diag.h"]:
            res = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{path}"],
                                 stdout=subprocess.PIPE, stderr=subprocess.PIPE)
            if res.returncode != 0:   # a file the revision does not have yet
                continue
            out = res.stdout
            dst = os.path.join(src_root, path)
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            old = open(dst, "rb").read() if os.path.exists(dst) else None
            if old != out:
                with open(dst, "wb") as f:
                    f.write(out)
        csrc = os.path.join(src_root, "sparsergps_amd", "csrc")
    return _build_into(outdir, os.path.join(outdir, "libsgp.so"), defs, force, verbose, csrc)


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        # variant NAME [REV] [-DFLAG ...]
        rest = sys.argv[3:]
        rev = rest.pop(0) if rest and not rest[0].startswith("-") else None
        print(build_variant(sys.argv[2], rest, verbose=True, rev=rev))
    else:
        print(build(force=True, verbose=True))
