"""Parity helpers: run the same seeded columnar batches through the device
engine (libsiddhi_hip) and the CPU oracle and compare the output streams.
Test infrastructure only."""
import numpy as np

from siddhi_amd import planner as pl
from siddhi_amd import query_compiler as qc
from siddhi_amd.runtime import ColumnBatch

from oracle_engine import OracleQueryEngine


def compile_single_query(app_text, dictionary=None, query_index=0):
    app = qc.parse(app_text)
    d = dictionary or pl.StringDictionary()
    item = app.execution_order[query_index]
    if isinstance(item, qc.Partition):
        return pl.plan_query(app, item.queries[0], d, item), d
    return pl.plan_query(app, item, d, None), d


def stock_batch(symbol, price, volume, ts, call_size=1024):
    n = len(ts)
    offs = np.arange(0, n, call_size, dtype=np.int64)
    offs = np.append(offs, np.int64(n))
    return ColumnBatch(ts, [symbol, price, volume], [None, None, None], offs)


def concat_rows(parts):
    if not parts:
        return (np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int64),
                np.zeros((0, 0), np.uint64), np.zeros((0, 0), np.uint8))
    return tuple(np.concatenate([p[k] for p in parts]) for k in range(5))


def run_oracle(qp, batches):
    """batches: list of (stream, ColumnBatch); each InputHandler call pushed separately."""
    eng = OracleQueryEngine(qp, None)
    parts = []
    cid = 0
    for si, b in batches:
        offs = b.call_offsets
        for c in range(len(offs) - 1):
            s, e = int(offs[c]), int(offs[c + 1])
            sub = ColumnBatch(b.ts[s:e], [x[s:e] for x in b.cols],
                              [None if x is None else x[s:e] for x in b.nulls])
            chunks = eng.set_time(int(b.ts[e - 1])) + eng.push(si, sub)
            for ch in chunks:
                n = len(ch.ts)
                parts.append((np.full(n, cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                cid += 1
    eng.close()
    return concat_rows(parts)


def run_device(qp, batches, exact=False):
    """exact: window aggregates as the bit-exact sequential fold (shd_set_option
    "exact_aggregates"); default: the product's segmented scans."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    dq = DeviceQuery(qp.ir)
    if exact and dq.engine_kind == 2:
        dq.set_option("exact_aggregates", 1)
    parts = []
    for si, b in batches:
        cols = [np.ascontiguousarray(c) for c in b.cols]
        nuls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in b.nulls]
        ts = np.ascontiguousarray(b.ts, np.int64)
        # playback time advances per InputHandler call inside the batch (advance_time)
        dq.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols],
                    [0 if x is None else x.ctypes.data for x in nuls], SHD_MEM_HOST,
                    b.call_offsets if len(b.call_offsets) > 2 else None, True)
        r = dq.poll()
        if r is not None:
            parts.append(r)
    counters = dq.counters()
    kind = dq.engine_kind
    dq.close()
    return concat_rows(parts), counters, kind


def chunk_boundaries(chunk_ids):
    if len(chunk_ids) == 0:
        return np.zeros(0, bool)
    return np.r_[True, chunk_ids[1:] != chunk_ids[:-1]]


def assert_same_rows(dev, ora, float_cols=(), rtol=0.0):
    dc, dt, dts, dv, dn = dev
    oc, ot, ots, ov, on = ora
    assert len(dts) == len(ots), "row count: device %d vs oracle %d" % (len(dts), len(ots))
    if len(dts) == 0:
        return
    np.testing.assert_array_equal(dt, ot)
    np.testing.assert_array_equal(dts, ots)
    np.testing.assert_array_equal(dn, on)
    np.testing.assert_array_equal(chunk_boundaries(dc), chunk_boundaries(oc))
    if rtol == 0.0:
        np.testing.assert_array_equal(dv, ov)
    else:
        for k in range(dv.shape[1]):
            if k in float_cols:
                a = dv[:, k].view(np.float64)
                b = ov[:, k].view(np.float64)
                np.testing.assert_allclose(a, b, rtol=rtol, atol=0)
            else:
                np.testing.assert_array_equal(dv[:, k], ov[:, k])


AGG_RTOL = 1e-9   # BASELINE.json north_star: double aggregates within 1e-9 relative


def float_cols(qp):
    """Output columns of double / float type (window aggregates)."""
    return tuple(i for i, t in enumerate(qp.output_types) if t in (3, 4))


def assert_rows_agg(dev, ora, qp, exact):
    """Window-aggregate outputs: bit-exact in exact mode; in segmented-scan mode
    every non-floating column, timestamp, null flag and callback boundary
    exact and floating columns within AGG_RTOL."""
    if exact:
        assert_same_rows(dev, ora)
    else:
        assert_same_rows(dev, ora, float_cols=float_cols(qp), rtol=AGG_RTOL)
