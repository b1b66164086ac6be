"""Device-code hygiene checks on the gfx950 assembly of libsiddhi_hip (CPU only).

* no vector-memory access may address the kernarg segment (those fault on the
  MI355X pool; argument blocks are passed through device memory instead);
* the hot kernels use no scratch (private segment) memory.
"""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from isa_check import scan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "siddhi_amd", "csrc")
SOURCES = ["engine_pattern.hip", "engine_single.hip", "engine_window.hip", "engine_nfa.hip", "primitives.hip",
           "engine_absent.hip", "route.hip"]


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa")
    hdrs = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    hdrs += [os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))]
    newest_input = max(os.path.getmtime(h) for h in hdrs)

    def one(src):
        # the build's own gfx950 assembly (Makefile: -save-temps=obj) when it is
        # newer than the source and every header
        kept = os.path.join(CSRC, "build", src.rsplit(".", 1)[0] + "-hip-amdgcn-amd-amdhsa-gfx950.s")
        if os.path.exists(kept) and os.path.getmtime(kept) >= max(newest_input,
                                                                  os.path.getmtime(os.path.join(CSRC, src))):
            return kept
        dst = str(out / (src + ".s"))
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-x", "hip",
                               "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", dst],
                              stderr=subprocess.DEVNULL)
        return dst

    with ThreadPoolExecutor(len(SOURCES)) as ex:
        return list(ex.map(one, SOURCES))


def test_no_vector_loads_from_kernarg_segment(asm):
    bad = []
    for p in asm:
        bad += scan(p)
    assert not bad, "\n".join("%s:%d %s" % (k[:60], ln, l) for k, ln, l in bad)


def test_hot_kernels_use_no_scratch(asm):
    text = "".join(open(p).read() for p in asm)
    kernels = re.findall(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.private_segment_fixed_size:\s+(\d+)", text)
    assert kernels
    for name, priv in kernels:
        if any(k in name for k in ("k_prepare", "k_forward_scan", "k_project", "k_filter", "k_fold", "k_emit")):
            assert int(priv) == 0, "%s uses %s bytes of scratch" % (name, priv)
