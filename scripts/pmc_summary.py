"""Per-stage HBM traffic and kernel time of the pattern engine from rocprofv3 output.

    python scripts/pmc_summary.py --trace <kernel_trace.csv> --fetch <FETCH_SIZE counter_collection.csv>
        --write <WRITE_SIZE counter_collection.csv> --events <events per push> --out profiles/rNN_pmc_P3.json

Kernels are assigned to the engine's stages (the names bench.py reports in
`stage_ms_per_step`) by walking the dispatch sequence of each push: a stage
starts at its marker kernel and runs until the next marker.  HBM bytes follow
MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE are KiB;
FETCH_SIZE counts half the bytes of a streaming read on gfx950, so it is
doubled; WRITE_SIZE is exact.  Each counter comes from its own --pmc pass
(they do not fit one pass).  Output: per stage, per push, and per event.
"""
import argparse
import csv
import json
from collections import defaultdict

def stage_sequence(names):
    """Stage of every dispatch (None for copies before the first push)."""
    out, stage = [], None
    for nm in names:
        if "k_prepare" in nm:
            stage = "prepare"
        elif "k_rs_hist" in nm and stage == "prepare":
            stage = "key_sort"
        elif "k_forward_scan" in nm:
            stage = "forward_scan"
        elif "k_scan_" in nm and stage == "forward_scan":
            stage = "compact"
        elif "k_emit_pairs" in nm:
            stage = "order_project"
        elif "k_gather_carry" in nm:
            stage = "carry"
        out.append(stage if "rocclr" not in nm else None)
    return out


def load_counter(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    names = [r["Kernel_Name"] for r in rows]
    vals = [float(r["Counter_Value"]) for r in rows]
    return names, vals


def per_stage(names, vals, scale):
    st = stage_sequence(names)
    pushes = sum(1 for nm in names if "k_prepare" in nm) or 1
    acc = defaultdict(float)
    for s, v in zip(st, vals):
        if s:
            acc[s] += v * scale
    return {k: v / pushes for k, v in acc.items()}, pushes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--events", type=int, required=True, help="events per push in the PMC runs")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    tr = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Dispatch_Id"]))
    tnames = [r["Kernel_Name"] for r in tr]
    tdur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in tr]
    t_stage, t_push = per_stage(tnames, tdur, 1.0)
    kern = defaultdict(lambda: [0, 0.0])
    for nm, d in zip(tnames, tdur):
        short = nm.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("shd::", "")
        kern[short][0] += 1
        kern[short][1] += d

    fn, fv = load_counter(a.fetch)
    wn, wv = load_counter(a.write)
    f_stage, f_push = per_stage(fn, fv, 2 * 1024.0)   # KiB, half-counted streaming reads on gfx950
    w_stage, w_push = per_stage(wn, wv, 1024.0)
    out = {
        "source": {"trace": a.trace, "fetch": a.fetch, "write": a.write},
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
        "pmc_events_per_push": a.events,
        "pmc_pushes": f_push,
        "trace_pushes": t_push,
        "stages": {},
        "kernels_us_avg": {k: round(v[1] / v[0] / 1e3, 1) for k, v in sorted(kern.items(), key=lambda x: -x[1][1])},
    }
    for s in sorted(set(f_stage) | set(w_stage) | set(t_stage)):
        rd, wr = f_stage.get(s, 0.0), w_stage.get(s, 0.0)
        out["stages"][s] = {
            "kernel_us_per_push": round(t_stage.get(s, 0.0) / 1e3, 1),
            "hbm_read_bytes_per_push": round(rd),
            "hbm_write_bytes_per_push": round(wr),
            "hbm_bytes_per_event": round((rd + wr) / a.events, 3),
        }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["stages"], indent=1))


if __name__ == "__main__":
    main()
