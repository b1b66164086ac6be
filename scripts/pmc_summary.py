"""Per-kernel HBM traffic and time of one bench command from rocprofv3 output.

    python scripts/pmc_summary.py --trace <kernel_trace.csv> --fetch <FETCH_SIZE counter_collection.csv>
        --write <WRITE_SIZE counter_collection.csv> --events <events per push> --pushes <pushes in the runs>
        --out profiles/rNN_pmc_<config>.json

HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE
are KiB; FETCH_SIZE counts half the bytes of a coalesced streaming read on
gfx950, so it is doubled for streaming kernels, and one 64-B request per random
access, which is what a gather moves, so gather kernels (GATHER below) take it
as is -- both calibrated by scripts/calib_fetch.hip
(profiles/r05_fetch_calibration.json); WRITE_SIZE is exact.  Each counter comes from its own --pmc pass of
the same command (they do not fit one pass).  Output, per kernel: dispatches
per push, average duration (kernel trace), HBM bytes per dispatch, bytes per
event and the kernel's own HBM rate and fraction of the 8 TB/s peak; plus the
per-push totals (all kernels of a push).
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siddhi_amd.buildinfo import source_hash  # noqa: E402

PEAK_GBS = 8000.0
# kernels whose reads are dominated by row gathers (FETCH_SIZE x1); every other
# kernel streams (x2).  k_resume_list: one lane per deferred walk, each from a
# random sorted position, with the walk's f2 operands gathered by row (its
# only streamed read is the list, 4 B per deferred walk)
GATHER = ("k_gather_list", "k_project", "k_emit_pairs", "k_gather_bpos", "k_xw_gather_u64", "k_xw_gather_u32",
          "k_resume_list")


def fetch_factor(kernel):
    return 1.0 if kernel.startswith(GATHER) else 2.0


def short(nm):
    s = nm.replace("(anonymous namespace)::", "").replace("void ", "").replace("shd::", "")
    return s.split("(")[0]


def load(path, value):
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        acc[k][0] += 1
        acc[k][1] += value(r)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--events", type=int, required=True, help="events per push")
    ap.add_argument("--pushes", type=int, required=True, help="pushes in each profiled run")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    dur = load(a.trace, lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fetch = load(a.fetch, lambda r: float(r["Counter_Value"]) * 1024.0 * fetch_factor(short(r["Kernel_Name"])))
    write = load(a.write, lambda r: float(r["Counter_Value"]) * 1024.0)
    kernels, tot_b, tot_us = {}, 0.0, 0.0
    for k in sorted(dur, key=lambda x: -dur[x][1]):
        n, ns = dur[k]
        fb = fetch[k][1] / fetch[k][0] if fetch[k][0] else 0.0
        wb = write[k][1] / write[k][0] if write[k][0] else 0.0
        us = ns / n / 1e3
        per_push = n / a.pushes
        kernels[k] = {
            "dispatches_per_push": round(per_push, 2),
            "avg_us": round(us, 2),
            "hbm_read_bytes": round(fb),
            "hbm_write_bytes": round(wb),
            "hbm_bytes_per_event": round((fb + wb) * per_push / a.events, 3),
            "hbm_gbs": round((fb + wb) / (us * 1e3), 1) if us > 0 else None,
            "hbm_frac": round((fb + wb) / (us * 1e3) / PEAK_GBS, 4) if us > 0 else None,
        }
        tot_b += (fb + wb) * per_push
        tot_us += us * per_push
    out = {
        # the libsiddhi_hip sources these counters were taken on (bench.py
        # uses the traffic only when its own tree hashes the same)
        "build": source_hash(),
        "source": {"trace": a.trace, "fetch": a.fetch, "write": a.write},
        "correction": ("FETCH_SIZE KiB x1024, x2 for streaming kernels (gfx950 half-count), x1 for the gather "
                       "kernels %s (one 64-B request per access); WRITE_SIZE KiB x1024; calibration: "
                       "profiles/r05_fetch_calibration.json" % (list(GATHER),)),
        "events_per_push": a.events,
        "pushes": a.pushes,
        "push": {"kernel_us": round(tot_us, 1), "hbm_bytes": round(tot_b),
                 "hbm_bytes_per_event": round(tot_b / a.events, 3)},
        "kernels": kernels,
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["push"]), json.dumps({k: v["hbm_bytes_per_event"] for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
