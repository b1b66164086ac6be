"""State persistence: SiddhiAppRuntime.snapshot()/restore(), persist()/
restoreLastRevision() with an InMemoryPersistenceStore
(C/SiddhiAppRuntimeImpl.java:677-745, C/util/snapshot/SnapshotService.java:90,333).

* The reference's own persistence tests
  (modules/siddhi-core/src/test/java/io/siddhi/core/managment/PersistenceTestCase.java
  persistenceTest1 :62-143 window, persistenceTest2 :145-230 count pattern,
  persistenceTest3 :232-293 no store) transcribed against the runtime API, on
  the CPU oracle (checker) and on the device (libsiddhi_hip).
* Device parity: a stream cut at a push boundary, the device state
  snapshotted, restored into a fresh query and the rest pushed there, must give
  exactly the rows of an uninterrupted device run and of the oracle, for the
  pattern engine (P3), the window engine (W2 length / time) and the NFA engine
  (S4 shapes, partitioned and not).
"""
import numpy as np
import pytest

from oracle_engine import OracleQueryEngine
from parity import (assert_rows_agg, assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle,
                    stock_batch)
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import (InMemoryPersistenceStore, NoPersistenceStoreException, QueryCallback,
                                SiddhiManager)


class _Collect(QueryCallback):
    def __init__(self):
        self.rows = []

    def receive(self, timestamp, inEvents, removeEvents):
        for e in inEvents or []:
            self.rows.append(list(e.getData()))


WINDOW_APP = ("@app:name('Test') define stream StockStream ( symbol string, price float, volume int );"
              "@info(name = 'query1') from StockStream[price>10]#window.length(10) "
              "select symbol, price, sum(volume) as totalVol insert into OutStream ")
COUNT_APP = ("@app:name('Test') define stream Stream1 (symbol string, price float, volume int); "
             "define stream Stream2 (symbol string, price float, volume int); "
             "@info(name = 'query1') from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
             "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
             "   e1[3].price as price1_3, e2.price as price2 insert into OutputStream ;")


def _manager(engine):
    return SiddhiManager(engine_factory=OracleQueryEngine) if engine == "oracle" else SiddhiManager()


def _persistence_test1(engine):
    """PersistenceTestCase.persistenceTest1 (:62-143): length window, persist, 2 lost events, restore."""
    m = _manager(engine)
    m.setPersistenceStore(InMemoryPersistenceStore())
    cb = _Collect()
    rt = m.createSiddhiAppRuntime(WINDOW_APP)
    rt.addCallback("query1", cb)
    ih = rt.getInputHandler("StockStream")
    rt.start()
    ih.send(["IBM", 75.6, 100])
    ih.send(["WSO2", 75.6, 100])
    assert cb.rows[-1][2] == 200
    rt.persist()
    ih.send(["IBM", 75.6, 100])
    ih.send(["WSO2", 75.6, 100])
    rt.shutdown()
    rt = m.createSiddhiAppRuntime(WINDOW_APP)
    rt.addCallback("query1", cb)
    ih = rt.getInputHandler("StockStream")
    rt.start()
    assert rt.restoreLastRevision() is not None
    ih.send(["IBM", 75.6, 100])
    ih.send(["WSO2", 75.6, 100])
    rt.shutdown()
    assert len(cb.rows) <= 6
    assert all(r[0] in ("IBM", "WSO2") for r in cb.rows)
    assert cb.rows[-1][2] == 400


def _persistence_test2(engine):
    """PersistenceTestCase.persistenceTest2 (:145-230): count pattern state survives a restart."""
    m = _manager(engine)
    m.setPersistenceStore(InMemoryPersistenceStore())
    cb = _Collect()
    rt = m.createSiddhiAppRuntime(COUNT_APP)
    rt.addCallback("query1", cb)
    s1 = rt.getInputHandler("Stream1")
    rt.start()
    s1.send(["WSO2", 25.6, 100])
    s1.send(["GOOG", 47.6, 100])
    s1.send(["GOOG", 13.7, 100])
    assert cb.rows == []
    rt.persist()
    rt.shutdown()
    rt = m.createSiddhiAppRuntime(COUNT_APP)
    rt.addCallback("query1", cb)
    s1, s2 = rt.getInputHandler("Stream1"), rt.getInputHandler("Stream2")
    rt.start()
    rt.restoreLastRevision()
    s2.send(["IBM", 45.7, 100])
    s1.send(["GOOG", 47.8, 100])
    s2.send(["IBM", 55.7, 100])
    rt.shutdown()
    assert len(cb.rows) == 1
    f32 = lambda x: float(np.float32(x))   # noqa: E731  (Java float values)
    assert cb.rows[0] == [f32(25.6), f32(47.6), None, None, f32(45.7)]


def _restore_after_new_symbol(engine):
    """a symbol interned between persist() and restoreLastRevision()
    on the same runtime (the live dictionary outgrew the snapshot's) must not
    make the restore fail; the window then holds the persisted events only."""
    m = _manager(engine)
    m.setPersistenceStore(InMemoryPersistenceStore())
    cb = _Collect()
    rt = m.createSiddhiAppRuntime(WINDOW_APP)
    rt.addCallback("query1", cb)
    ih = rt.getInputHandler("StockStream")
    rt.start()
    ih.send(["IBM", 75.6, 100])
    rt.persist()
    ih.send(["ORCL", 75.6, 100])    # new string after the snapshot
    assert cb.rows[-1][2] == 200
    assert rt.restoreLastRevision() is not None
    ih.send(["ORCL", 75.6, 100])
    assert cb.rows[-1] == ["ORCL", float(np.float32(75.6)), 200]
    rt.shutdown()


def test_restore_after_new_symbol_oracle():
    _restore_after_new_symbol("oracle")


@pytest.mark.gpu
def test_restore_after_new_symbol_device(hip_available):
    _restore_after_new_symbol("device")


def test_send_batch_requires_start():
    """the columnar path refuses events before start(), like send()."""
    from siddhi_amd.runtime import ColumnBatch
    m = SiddhiManager(engine_factory=OracleQueryEngine)
    rt = m.createSiddhiAppRuntime(WINDOW_APP)
    b = ColumnBatch(np.array([1], np.int64), [np.array([0], np.uint32), np.array([11.0], np.float32),
                                              np.array([1], np.int32)], [None, None, None])
    with pytest.raises(RuntimeError):
        rt.getInputHandler("StockStream").send_batch(b)


def test_persistence_window_oracle():
    _persistence_test1("oracle")


def test_persistence_count_pattern_oracle():
    _persistence_test2("oracle")


def test_persist_without_store_raises():
    """PersistenceTestCase.persistenceTest3 (:232-293): NoPersistenceStoreException."""
    m = SiddhiManager(engine_factory=OracleQueryEngine)
    rt = m.createSiddhiAppRuntime(COUNT_APP)
    rt.start()
    with pytest.raises(NoPersistenceStoreException):
        rt.persist()


def test_restore_rejects_other_app():
    m = SiddhiManager(engine_factory=OracleQueryEngine)
    a = m.createSiddhiAppRuntime(WINDOW_APP)
    b = m.createSiddhiAppRuntime(COUNT_APP)
    from siddhi_amd.runtime import CannotRestoreSiddhiAppStateException
    with pytest.raises(CannotRestoreSiddhiAppStateException):
        b.restore(a.snapshot())


@pytest.mark.gpu
def test_persistence_window_device(hip_available):
    _persistence_test1("device")


@pytest.mark.gpu
def test_persistence_count_pattern_device(hip_available):
    _persistence_test2("device")


def _split(sym, price, vol, ts, parts, call=1024):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])]


def _run_with_restore(qp, batches, cut):
    """Device: batches[:cut] on one query, snapshot, restore into a fresh query, batches[cut:]."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    parts = []

    def feed(dq, bs):
        for si, b in bs:
            cols = [np.ascontiguousarray(c) for c in b.cols]
            ts = np.ascontiguousarray(b.ts, np.int64)
            dq.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols], [0] * len(cols), SHD_MEM_HOST,
                        b.call_offsets if len(b.call_offsets) > 2 else None, True)
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
    return concat_rows(parts)


RESTORE_CASES = [
    ("P3", wl.P3_APP, 200_000, 20_000, 0.01, 4),
    ("P3-dense", wl.P3_APP, 120_000, 3_000, 1e-4, 3),
    ("W2-length", wl.W2_LENGTH_APP, 100_000, 1000, 0.1, 4),
    ("W2-time", wl.W2_TIME_APP, 100_000, 1000, 0.5, 4),
    ("S4-or", wl.S4_APPS["or"], 30_000, 100, 1.0, 3),
    # window lanes: the carried tail events
    ("S4-seq-window", wl.S4_APPS["seq"].replace("<2:5>", "<1:3>"), 30_000, 100, 1.0, 4),
    ("S4-seqplus-part", wl.S4_PART_APPS["seqplus"], 30_000, 50, 1.0, 3),
    ("S4-and-part", wl.S4_PART_APPS["and"], 30_000, 100, 1.0, 3),
    # half-filled AND partials carry their operand event through the snapshot
    ("S4-and-wide", wl.S4_APPS["and"].replace("price>e1.price*1.2", "price>e1.price*1.3")
     .replace("within 1 sec", "within 40 milliseconds"), 30_000, 100, 1.0, 3),
    ("S4-not-part", wl.S4_PART_APPS["not"], 30_000, 100, 1.0, 3),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,app,n,keys,delta,parts", RESTORE_CASES, ids=[c[0] for c in RESTORE_CASES])
def test_device_snapshot_restore_midstream(hip_available, name, app, n, keys, delta, parts):
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=301)
    batches = _split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    whole, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    exact = not name.startswith("W2")   # W2: segmented-scan aggregates (1e-9 relative)
    assert_rows_agg(whole, ora, qp, exact)
    for cut in range(1, len(batches)):
        restored = _run_with_restore(qp, batches, cut)
        assert_rows_agg(restored, ora, qp, exact)
        if not exact:   # restoring mid-stream changes nothing in the device's own results
            assert_same_rows(restored, whole)


@pytest.mark.gpu
def test_restore_rejects_other_plan(hip_available):
    from siddhi_amd.hip_engine import DeviceQuery, SiddhiHipError
    qa, _ = compile_single_query(wl.P3_APP)
    qb, _ = compile_single_query(wl.W2_LENGTH_APP)
    a, b = DeviceQuery(qa.ir), DeviceQuery(qb.ir)
    try:
        with pytest.raises(SiddhiHipError):
            b.restore(a.snapshot())
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_snapshot_restore_sparse_key_carry(hip_available):
    """A snapshot taken while the pattern engine carries the open partials of
    sparse keys (P3 shape) restores them; the rest of the stream then gives
    the oracle's rows."""
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(200_000, 20_000, 0.05, seed_offset=307)
    batches = _split(sym, price, vol, ts, 4)
    ora = run_oracle(qp, batches)
    assert len(ora[2]) > 0
    for cut in range(1, len(batches)):
        assert_same_rows(_run_with_restore(qp, batches, cut), ora)


# ---- output rate limiters across persist() / restoreRevision()
# The limiters' RateLimiterState maps (counter, held rows, per-group maps,
# scheduled time) ride in the snapshot head: an uninterrupted run and a run
# restored into a fresh runtime mid-stream emit the same callback chunks.
RATE_APPS = {
    "every-3-events": "output every 3 events",
    "last-every-4-events-grouped": "output last every 4 events",
    "first-every-5-events-grouped": "output first every 5 events",
    "all-every-time": "output all every 100 milliseconds",
    "last-every-time-grouped": "output last every 50 milliseconds",
}


def _rate_app(rate, grouped):
    return ("@app:name('R') @app:playback define stream S (symbol string, price double, volume long); "
            "@info(name = 'q') from S select symbol, price, volume %s %s insert into O;"
            % ("group by symbol" if grouped else "", rate))


def _rate_run(app, events, cut=None):
    """Callback chunks of `app` over `events` (ts, data); with `cut`, persist
    after event cut - 1 and continue in a restored fresh runtime."""
    m = SiddhiManager(engine_factory=OracleQueryEngine)
    m.setPersistenceStore(InMemoryPersistenceStore())
    chunks = []

    class C(QueryCallback):
        def receive(self, timestamp, inEvents, removeEvents):
            chunks.append([(e.getTimestamp(), list(e.getData())) for e in inEvents or []])

    rt = m.createSiddhiAppRuntime(app)
    rt.clock = lambda: 1000   # the timed limiters schedule from the wall clock (partitionCreated)
    rt.addCallback("q", C())
    rt.start()
    ih = rt.getInputHandler("S")
    for k, (ts, d) in enumerate(events):
        if cut is not None and k == cut:
            rev = rt.persist().getRevision()
            rt.shutdown()
            rt = m.createSiddhiAppRuntime(app)
            rt.clock = lambda: 5000   # a later wall clock: the restored schedule must win
            rt.addCallback("q", C())
            rt.start()
            rt.restoreRevision(rev)
            ih = rt.getInputHandler("S")
        ih.send(ts, d)
    rt.shutdown()
    return chunks


@pytest.mark.parametrize("name", list(RATE_APPS))
def test_rate_limiter_state_survives_restore(name):
    grouped = name.endswith("grouped")
    app = _rate_app(RATE_APPS[name], grouped)
    rng = np.random.default_rng(7)
    events = [(1000 + 7 * k, ["S%d" % int(rng.integers(0, 4)), float(rng.integers(50, 100)), k]) for k in range(60)]
    whole = _rate_run(app, events)
    assert sum(len(c) for c in whole) > 0
    for cut in (1, 7, 23, 41):
        assert _rate_run(app, events, cut) == whole, cut
