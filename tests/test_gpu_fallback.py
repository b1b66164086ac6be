"""Inputs the pattern forward scan cannot process on its own formulation but
the reference accepts: per-key timestamp regressions under `within`
(StreamPreStateProcessor.isExpired uses Math.abs and expireEvents breaks at
the first non-expired partial, ST/StreamPreStateProcessor.java:118-129,326-361).
The query hands its open partials over to the device's generic NFA engine
(replay of the events that created them) and continues there; results must
equal the oracle row for row.  Without `within` a regression changes nothing
and the forward scan keeps the query."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu


def _regress(ts, rng, frac=0.02, back=3):
    """Move a fraction of events back in time by up to `back` ms (per-key order broken)."""
    ts = ts.copy()
    idx = rng.choice(len(ts), int(len(ts) * frac), replace=False)
    ts[idx] -= rng.integers(1, back + 1, len(idx))
    return ts


@pytest.mark.parametrize("partitioned", [True, False])
@pytest.mark.parametrize("where", ["first", "later"])
def test_time_regression_hands_over_to_nfa(hip_available, partitioned, where):
    app = wl.P3_APP if partitioned else wl.P1_APP
    qp, _ = compile_single_query(app.replace("within 1 sec", "within 6 milliseconds"))
    rng = np.random.default_rng(31 + partitioned)
    n, keys = 12_000, 300 if partitioned else 40
    sym, price, vol, ts = wl.stock_stream(n, keys, 0.05, seed_offset=5)
    cuts = [0, 4000, 8000, n]
    bad = 0 if where == "first" else 1
    batches = []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        t = _regress(ts[a:b], rng) if i == bad else ts[a:b]
        batches.append((0, stock_batch(sym[a:b], price[a:b], vol[a:b], t, 1000)))
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert kind == 4   # the query continued on the generic NFA engine
    assert counters["events"] == n


def test_no_within_regression_stays_on_forward_scan(hip_available):
    """without `within` timestamps cannot change which partial
    completes; a decreasing key clock must neither fail nor leave the forward scan."""
    app = ("@app:playback define stream S (k int, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>60] -> e2=S[p>e1.p*1.1] "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(9)
    n = 20_000
    k = rng.integers(0, 500, n).astype(np.int32)
    p = rng.uniform(0, 100, n)
    ts = 5_000_000 - np.arange(n, dtype=np.int64)   # time runs backwards
    batches = [(0, ColumnBatch(ts[a:b], [k[a:b], p[a:b]], [None, None], np.arange(a, b + 1, 500) - a))
               for a, b in ((0, 9000), (9000, n))]
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert kind == 1


@pytest.mark.parametrize("partitioned", [True, False])
@pytest.mark.parametrize("where", ["first", "later"])
def test_and_regression_hands_over_half_filled_partials(hip_available, partitioned, where):
    """every e1 -> e2 and e3: partials holding one operand when timestamps go
    back are handed over with that operand's event (replayed past the start
    state when its own partial is gone); the continuation equals the oracle."""
    apps = wl.S4_PART_APPS if partitioned else wl.S4_APPS
    qp, _ = compile_single_query(apps["and"].replace("within 1 sec", "within 40 milliseconds")
                                 .replace("e1.price*1.2", "e1.price*1.02").replace("e1.price*0.8", "e1.price*0.98"))
    rng = np.random.default_rng(71 + partitioned)
    n, keys = 12_000, 60 if partitioned else 20
    sym, price, vol, ts = wl.stock_stream(n, keys, 0.2, seed_offset=6)
    cuts = [0, 4000, 8000, n]
    bad = 1 if where == "first" else 2
    batches = []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        t = _regress(ts[a:b], rng, frac=0.01, back=5) if i == bad else ts[a:b]
        batches.append((0, stock_batch(sym[a:b], price[a:b], vol[a:b], t, 1000)))
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert kind == 4
    assert counters["events"] == n


@pytest.mark.parametrize("app", [wl.P3_APP, wl.P1_APP], ids=["P3", "P1"])
def test_snapshot_after_hand_over_restores_into_fresh_query(hip_available, app):
    """A query that switched engines snapshots the NFA engine's state; restoring
    it into a freshly loaded query (which starts on the forward scan) switches
    that query too, and the continuation equals the oracle."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query(app.replace("within 1 sec", "within 6 milliseconds"))
    rng = np.random.default_rng(4)
    sym, price, vol, ts = wl.stock_stream(9000, 200, 0.05, seed_offset=8)
    t1 = _regress(ts[:4000], rng)
    batches = [(0, stock_batch(sym[:4000], price[:4000], vol[:4000], t1, 1000)),
               (0, stock_batch(sym[4000:], price[4000:], vol[4000:], ts[4000:], 1000))]
    ora = run_oracle(qp, batches)

    def push(dq, b):
        cols = [np.ascontiguousarray(c) for c in b.cols]
        t = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(0, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0] * 3, SHD_MEM_HOST,
                    b.call_offsets, True)
        return dq.poll()

    a = DeviceQuery(qp.ir)
    fresh = DeviceQuery(qp.ir)
    try:
        parts = [r for r in [push(a, batches[0][1])] if r is not None]
        image = a.snapshot()
        assert fresh.engine_kind == 1
        fresh.restore(image)
        r = push(fresh, batches[1][1])
        if r is not None:
            parts.append(r)
        assert fresh.engine_kind == 4
    finally:
        a.close()
        fresh.close()
    assert_same_rows(concat_rows(parts), ora)
