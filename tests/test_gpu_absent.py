"""Absent forward-scan engine (engine_absent.hip) for config S4's
`every e1=StockStream[price>98] -> not StockStream[price>e1.price] for 1 sec`
vs the CPU oracle (AbsentStreamPreStateProcessor + playback timers): every
row, timestamp and callback chunk identical, across micro-batch splits, call
sizes, clock moves between pushes (shd_set_time), a snapshot / restore, and a
push whose time goes back (hand-over to the generic NFA engine)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

ENGINE_PATTERN, ENGINE_NFA = 1, 4
APP = wl.S4_APPS["not"]


def split(sym, price, vol, ts, parts, call):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])
            if b > a]


@pytest.mark.parametrize("parts", [1, 3, 7])
@pytest.mark.parametrize("call", [1, 37, 1024])
def test_absent_equals_oracle(hip_available, parts, call):
    qp, _ = compile_single_query(APP)
    n = 20000 if call > 1 else 6000
    sym, price, vol, ts = wl.stock_stream(n, 1000, 1.0, seed_offset=5 + parts)
    batches = split(sym, price, vol, ts, parts, call)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("delta", [2.0, 20.0])
def test_absent_time_scales(hip_available, delta):
    """Calls spanning half a deadline and calls spanning many deadlines (every
    call's clock move fires several timers at once)."""
    qp, _ = compile_single_query(APP)
    sym, price, vol, ts = wl.stock_stream(30000, 1000, delta, seed_offset=9)
    batches = split(sym, price, vol, ts, 4, 256)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN and len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_absent_clock_moves_between_pushes(hip_available):
    """shd_set_time between pushes fires the carried partials it reaches
    (before the next event), like the oracle's set_time."""
    from oracle_engine import OracleQueryEngine
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query(APP)
    sym, price, vol, ts = wl.stock_stream(12000, 1000, 1.0, seed_offset=13)
    batches = split(sym, price, vol, ts, 6, 512)
    eng = OracleQueryEngine(qp, None)
    dq = DeviceQuery(qp.ir)
    ora_parts, dev_parts, cid = [], [], 0
    for k, (si, b) in enumerate(batches):
        offs = b.call_offsets
        for c in range(len(offs) - 1):
            s0, e0 = int(offs[c]), int(offs[c + 1])
            sub = ColumnBatch(b.ts[s0:e0], [x[s0:e0] for x in b.cols], [None for _ in b.cols])
            for ch in eng.set_time(int(b.ts[e0 - 1])) + eng.push(si, sub):
                ora_parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                cid += 1
        cols = [np.ascontiguousarray(x) for x in b.cols]
        t = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(si, b.n, t.ctypes.data, [x.ctypes.data for x in cols], [0, 0, 0], SHD_MEM_HOST, b.call_offsets,
                    True)
        # a clock move between pushes: half a deadline on
        tmove = int(b.ts[-1]) + 500 + 100 * k
        for ch in eng.set_time(tmove):
            ora_parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
            cid += 1
        dq.set_time(tmove)
        r = dq.poll()
        if r is not None:
            dev_parts.append(r)
    eng.close()
    kind = dq.engine_kind
    dq.close()
    assert kind == ENGINE_PATTERN
    ora, dev = concat_rows(ora_parts), concat_rows(dev_parts)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_absent_time_going_back_hands_over(hip_available):
    """A push whose events go back in time continues on the generic NFA engine
    with the open partials replayed; rows equal the oracle's."""
    qp, _ = compile_single_query(APP)
    sym, price, vol, ts = wl.stock_stream(12000, 1000, 1.0, seed_offset=17)
    batches = split(sym, price, vol, ts, 3, 1024)
    batches.append(batches[1])
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == ENGINE_NFA
    assert_same_rows(dev, ora)


def test_absent_snapshot_restore(hip_available):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query(APP)
    sym, price, vol, ts = wl.stock_stream(16000, 1000, 1.0, seed_offset=19)
    batches = split(sym, price, vol, ts, 4, 1024)
    ora = run_oracle(qp, batches)
    for cut in range(1, 4):
        parts = []

        def feed(dq, bs):
            for si, b in bs:
                cols = [np.ascontiguousarray(c) for c in b.cols]
                t = np.ascontiguousarray(b.ts, np.int64)
                dq.push_raw(si, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0, 0, 0], SHD_MEM_HOST,
                            b.call_offsets, True)
                r = dq.poll()
                if r is not None:
                    parts.append(r)
        dq = DeviceQuery(qp.ir)
        feed(dq, batches[:cut])
        image = dq.snapshot()
        dq.close()
        dq2 = DeviceQuery(qp.ir)
        dq2.restore(image)
        feed(dq2, batches[cut:])
        dq2.close()
        assert_same_rows(concat_rows(parts), ora)


def test_absent_scan_off_equals(hip_available, monkeypatch):
    monkeypatch.setenv("SHD_NO_ABSENT_SCAN", "1")
    qp, _ = compile_single_query(APP)
    sym, price, vol, ts = wl.stock_stream(8000, 1000, 1.0, seed_offset=23)
    batches = split(sym, price, vol, ts, 2, 1024)
    dev, _, kind = run_device(qp, batches)
    assert kind == ENGINE_NFA
    assert_same_rows(dev, run_oracle(qp, batches))
