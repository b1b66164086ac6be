"""Diagnostic (GPU): tiny P3 repros of the time-back hand-over -- one key's
events of push 0, then the same events again (time goes back: the pattern
engine hands its open partials to the NFA engine).  Variant "emu": the replay
emulated by plain events (a stabilize-only event = an event that passes no
filter) pushed to the NFA engine directly.  Prints device vs oracle rows."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from parity import compile_single_query, run_device, run_oracle, stock_batch  # noqa: E402
from siddhi_amd import workloads as wl  # noqa: E402


def rows(r):
    return [(int(t), int(v[0]), round(float(v[1:2].view(np.float64)[0]), 4), round(float(v[2:3].view(np.float64)[0]), 4))
            for t, v in zip(r[2], r[3])]


def main():
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(300_000, 100_000, 0.05, seed_offset=41)
    n0 = 100_000 // 1024 * 1024
    keys = [257] + [int(k) for k in np.unique(sym[:n0])[:40]]
    bad = 0
    for k in keys:
        idx = np.nonzero(sym[:n0] == k)[0]
        if len(idx) < 2:
            continue
        b0 = stock_batch(sym[idx], price[idx], vol[idx], ts[idx], 1)
        batches = [(0, b0), (0, b0)]
        ora = run_oracle(qp, batches)
        dev, _, kind = run_device(qp, batches)
        same = rows(dev) == rows(ora)
        if not same or k == 257:
            print("key %d kind %d events %s" % (k, kind, [(int(ts[i]) - 1700000000000, round(float(price[i]), 2)) for i in idx]))
            print("   dev", rows(dev))
            print("   ora", rows(ora))
        bad += 0 if same else 1
    print("differing keys:", bad, flush=True)


if __name__ == "__main__":
    main()
