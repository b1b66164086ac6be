"""The C-ABI library builds for gfx950, loads, and exports every entry point
include/siddhi_hip.h declares.  No compute calls (CPU only)."""
import ctypes
import os
import re

from siddhi_amd import hip_engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(shd_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("shd_ctx_create", "shd_plan_load", "shd_push", "shd_poll", "shd_set_time", "shd_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = hip_engine.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), "missing export %s" % s
    assert sorted(hip_engine.EXPORTED) == declared_symbols()


def test_library_is_gfx950_code_object():
    data = open(hip_engine.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_is_reported_cleanly():
    lib = hip_engine.load_library()
    n = ctypes.c_int(-1)
    assert lib.shd_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    if n.value == 0:
        ctx = ctypes.c_void_p()
        rc = lib.shd_ctx_create(None, 0, ctypes.byref(ctx))
        assert rc == hip_engine.SHD_E_DEVICE
        assert b"device" in lib.shd_last_error()


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors of shd_batch / shd_out / shd_counters (hip_engine.py)
    have the header's field offsets and sizes (compiled with the host C
    compiler against include/siddhi_hip.h), including the fields SURVEY.md §8b
    names: shd_out.state_idx, shd_out.in_seq, shd_batch.base_seq."""
    import subprocess
    fields = {"shd_batch": [f[0] for f in hip_engine.ShdBatch._fields_],
              "shd_out": [f[0] for f in hip_engine.ShdOut._fields_],
              "shd_counters": [f[0] for f in hip_engine.ShdCounters._fields_]}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "siddhi_hip.h"', 'int main(void) {']
    for st, fs in fields.items():
        src.append('printf("%s size %%zu\\n", sizeof(%s));' % (st, st))
        for f in fs:
            src.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (st, f, st, f))
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)])
    got = dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)]).decode().splitlines())
    for st, cls in (("shd_batch", hip_engine.ShdBatch), ("shd_out", hip_engine.ShdOut),
                    ("shd_counters", hip_engine.ShdCounters)):
        assert int(got["%s size" % st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(got["%s.%s" % (st, f)]) == getattr(cls, f).offset, (st, f)
    assert "state_idx" in fields["shd_out"] and "base_seq" in fields["shd_batch"]
