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
