"""Build hygiene (CPU): the product library is rebuilt whenever its compile flags change, the
product build refuses environment -D flags, and experiment knobs need a variant build."""
import os
import subprocess

import pytest

from sparsergps_amd import _build as B


def test_product_build_refuses_env_defs(monkeypatch):
    monkeypatch.setenv("SGP_HIPCC_DEFS", "-DSGP_CON_IL_PAT=3")
    with pytest.raises(RuntimeError, match="SGP_HIPCC_DEFS"):
        B.build()


def test_changed_define_forces_rebuild(tmp_path, monkeypatch):
    """A stamp written for other flags (an A/B build left in place) makes every object stale."""
    B.build()
    assert not B.stale()
    objs, todo = B._plan(B.LIBDIR, ())
    assert todo == []
    # the same objects judged against a different define: all stale
    _, todo_def = B._plan(B.LIBDIR, ("-DSGP_CON_IL_PAT=3",))
    assert [s for s, _ in todo_def] == B.SOURCES
    # an object whose stamp records an experiment define is rebuilt by the product build
    obj = objs[0]
    key = B._read_stamp(obj)
    try:
        B._write_stamp(obj, B._obj_key(B.SOURCES[0], ("-DSGP_CON_IL_PAT=3",)))
        assert B.stale()
        _, todo = B._plan(B.LIBDIR, ())
        assert [s for s, _ in todo] == [B.SOURCES[0]]
    finally:
        B._write_stamp(obj, key)
    assert not B.stale()


def test_library_stamp_covers_link(monkeypatch):
    B.build()
    lib_key = B._read_stamp(B.LIB)
    try:
        B._write_stamp(B.LIB, lib_key + "\0-DX")
        assert B.stale()
    finally:
        B._write_stamp(B.LIB, lib_key)
    assert not B.stale()


def test_stamps_are_path_independent():
    """The GPU box receives the tree at another path: the stamps must not name it."""
    B.build()
    for p in os.listdir(B.LIBDIR):
        if p.endswith(".cmd"):
            text = open(os.path.join(B.LIBDIR, p)).read()
            assert B.ROOT not in text and "hipcc" not in text


@pytest.mark.parametrize("knob", ["SGP_CON_IL_PAT=3", "SGP_LAP_RS_CFG=1", "SGP_CON_SHMEM=1"])
def test_experiment_knobs_need_probe_build(knob):
    src = os.path.join(B.CSRC, "sgp_probe.h")
    cmd = [B.hipcc(), "-x", "hip", "--offload-arch=gfx950", "-fsyntax-only", f"-D{knob}", src]
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    assert res.returncode != 0 and b"SGP_PROBE_BUILD" in res.stdout
    ok = subprocess.run(cmd + ["-DSGP_PROBE_BUILD"], stdout=subprocess.PIPE,
                        stderr=subprocess.STDOUT)
    assert ok.returncode == 0, ok.stdout.decode(errors="replace")


def test_ab_lib_must_be_a_variant(monkeypatch):
    from sparsergps_amd import _lib
    monkeypatch.setenv("SGP_AB_LIB", B.LIB)
    with pytest.raises(RuntimeError, match="tools"):
        _lib._ab_lib()
    monkeypatch.setenv("SGP_AB_LIB", os.path.join(B.VARIANT_ROOT, "x", "libsgp.so"))
    assert _lib._ab_lib().endswith(os.path.join("x", "libsgp.so"))
