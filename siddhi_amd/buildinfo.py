"""Identity of the libsiddhi_hip build a measurement was taken on.

`source_hash()` digests every source libsiddhi_hip.so is compiled from
(siddhi_amd/csrc/*.hip|*.h|*.cpp|Makefile and include/*.h).  PMC summaries
(scripts/pmc_summary.py) record it; bench.py only attaches a summary's HBM
traffic to its roofline when the hash equals the running tree's, so a bench
line never carries bytes measured on other code.
"""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files():
    pats = ["siddhi_amd/csrc/*.hip", "siddhi_amd/csrc/*.h", "siddhi_amd/csrc/*.cpp", "siddhi_amd/csrc/Makefile",
            "include/*.h"]
    out = []
    for p in pats:
        out.extend(glob.glob(os.path.join(ROOT, p)))
    return sorted(set(out))


def source_hash():
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(b"\0")
        with open(f, "rb") as fp:
            h.update(fp.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
