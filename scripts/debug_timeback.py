"""Diagnostic (GPU): P3 pushes whose last push goes back in time -- where do
the device and the oracle part?  Prints, per variant, the first differing row
with its in_seq.  Not a test; run by hand on the GPU box."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from parity import compile_single_query, run_oracle, stock_batch  # noqa: E402
from siddhi_amd import workloads as wl  # noqa: E402


def split(sym, price, vol, ts, parts, call=1024):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])]


def device_rows(qp, batches):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    dq = DeviceQuery(qp.ir)
    out = []
    for si, b in batches:
        cols = [np.ascontiguousarray(c) for c in b.cols]
        t = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(si, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0] * 3, SHD_MEM_HOST, b.call_offsets, True)
        r = dq.poll(with_seq=True)
        out.append((r, dq.engine_kind))
    dq.close()
    return out


def compare(name, qp, batches):
    ora = run_oracle(qp, batches)
    dev = device_rows(qp, batches)
    rows = [r for r, _ in dev if r is not None]
    kinds = [k for _, k in dev]
    dts = np.concatenate([r[2] for r in rows]) if rows else np.zeros(0)
    dv = np.concatenate([r[3] for r in rows]) if rows else np.zeros((0, 3))
    dseq = np.concatenate([r[5] for r in rows]) if rows else np.zeros(0)
    ots, ov = ora[2], ora[3]
    print("%-28s kinds %s rows dev %d ora %d" % (name, kinds, len(dts), len(ots)), flush=True)
    m = min(len(dts), len(ots))
    bad = np.nonzero((dts[:m] != ots[:m]) | np.any(dv[:m] != ov[:m], axis=1))[0]
    if len(bad) or len(dts) != len(ots):
        i = int(bad[0]) if len(bad) else m
        lo = max(0, i - 2)
        print("  first difference at row %d (device in_seq %s)" % (i, dseq[lo:i + 3]))
        for j in range(lo, min(i + 3, max(len(dts), len(ots)))):
            d = (dts[j], [int(x) for x in dv[j]]) if j < len(dts) else None
            o = (ots[j], [int(x) for x in ov[j]]) if j < len(ots) else None
            print("   row %d dev %s ora %s" % (j, d, o))
        # decode: value columns symbol id, p1 bits, p2 bits
        if i < len(ots):
            print("  oracle row symbol %d p1 %r p2 %r" % (ov[i][0], ov[i][1:2].view(np.float64)[0],
                                                       ov[i][2:3].view(np.float64)[0]))


def key_story(qp, batches, key):
    """Every event of one key and every output row of it, device and oracle."""
    seq = 0
    for j, (_, b) in enumerate(batches):
        for i in np.nonzero(b.cols[0] == key)[0]:
            print("  push %d seq %d ts %d price %.4f" % (j, seq + i, b.ts[i], b.cols[1][i]))
        seq += b.n
    ora = run_oracle(qp, batches)
    for r in range(len(ora[2])):
        if ora[3][r][0] == key:
            print("  ora row ts %d p1 %.4f p2 %.4f" % (ora[2][r], ora[3][r][1:2].view(np.float64)[0],
                                                    ora[3][r][2:3].view(np.float64)[0]))
    for r, _ in device_rows(qp, batches):
        if r is None:
            continue
        for q in range(len(r[2])):
            if r[3][q][0] == key:
                print("  dev row ts %d p1 %.4f p2 %.4f in_seq %d" % (r[2][q], r[3][q][1:2].view(np.float64)[0],
                                                                  r[3][q][2:3].view(np.float64)[0], r[5][q]))


def main():
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(300_000, 100_000, 0.05, seed_offset=41)
    b3 = split(sym, price, vol, ts, 3)
    compare("three pushes", qp, b3)
    later = b3[0][1]
    shifted = stock_batch(later.cols[0], later.cols[1], later.cols[2], later.ts + 100_000, 1024)
    compare("fourth push later in time", qp, b3 + [(0, shifted)])
    compare("fourth push back in time", qp, b3 + [b3[0]])
    key_story(qp, b3 + [b3[0]], 257)
    os.environ["SHD_FORCE_NFA"] = "1"
    compare("NFA only, back in time", qp, b3 + [b3[0]])


if __name__ == "__main__":
    main()
