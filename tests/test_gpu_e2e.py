"""The public API end to end on the device: SiddhiManager ->
InputHandler.send_batch (several InputHandler calls per batch) ->
QueryCallback / StreamCallback, against the same app on the CPU oracle
engine, which takes one call at a time.  With no query feeding another and
no rate limiter, the runtime hands a multi-call batch to each engine as ONE
push (SiddhiAppRuntime._batch_push_ok: the engine advances playback time per
call itself); every callback invocation -- its rows, timestamps, expired
flags and boundaries -- must be the per-call path's.  Also the vectorised
output decode (runtime.decode_columns) on every attribute type, nulls
included, and the per-call path the runtime keeps when a query is chained.

Reference: C/stream/input/InputHandler.java:85-95 (setCurrentTimestamp per
call), C/query/output/callback/QueryCallback.java:61-91."""
import math

import numpy as np
import pytest

from oracle_engine import OracleQueryEngine
from siddhi_amd import runtime as rt
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu


def record(app, sends, engine_factory, queries=None, streams=()):
    mgr = rt.SiddhiManager(engine_factory=engine_factory) if engine_factory else rt.SiddhiManager()
    r = mgr.createSiddhiAppRuntime(app)
    # symbol columns hold dictionary ids: intern S0000000.. so both runs decode them alike
    nk = max([int(b.cols[0].max()) + 1 for sid, b in sends if sid == "StockStream"] or [0])
    for i in range(nk):
        r.dictionary.id("S%07d" % i)
    got = {}
    for q in (queries or [x.name for x in r.queries]):
        got[q] = []
        r.addCallback(q, rt._FnQueryCallback(
            lambda ts, cur, rem, q=q: got[q].append(
                (ts, [(e.timestamp, e.data) for e in (cur or [])], [(e.timestamp, e.data) for e in (rem or [])]))))
    for sname in streams:
        got["#" + sname] = []
        r.addCallback(sname, rt._FnStreamCallback(
            lambda evs, sname=sname: got["#" + sname].append([(e.timestamp, e.data) for e in evs])))
    r.start()
    for sid, batch in sends:
        r.getInputHandler(sid).send_batch(batch)
    r.shutdown()
    return got


def stock(n, keys, delta, seed=0, call=1024, nulls=False):
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=seed)
    nm = [None, None, None]
    if nulls:
        rng = np.random.default_rng(seed)
        nm = [None, (rng.random(n) < 0.05).astype(np.uint8), (rng.random(n) < 0.05).astype(np.uint8)]
    offs = np.append(np.arange(0, n, call, dtype=np.int64), np.int64(n))
    return rt.ColumnBatch(ts, [sym, price, vol], nm, offs)


def same(a, b):
    """Equal callback payloads; doubles within the north_star's 1e-9 relative
    tolerance (window sums / averages come from the segmented scans)."""
    if isinstance(a, float) and isinstance(b, float):
        return a == b or math.isclose(a, b, rel_tol=1e-9, abs_tol=0.0)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    return a == b


def check(app, sends, queries=None, streams=()):
    dev = record(app, sends, None, queries, streams)
    ora = record(app, sends, OracleQueryEngine, queries, streams)
    assert dev.keys() == ora.keys()
    total = 0
    for k in ora:
        assert len(dev[k]) == len(ora[k]), k
        for a, b in zip(dev[k], ora[k]):
            assert same(a, b), (k, a, b)
        total += len(ora[k])
    assert total > 0
    return dev


def test_e2e_partitioned_pattern(hip_available):
    check(wl.P3_APP, [("StockStream", stock(60_000, 2_000, 0.5, seed=3))])


def test_e2e_windows_with_nulls(hip_available):
    app = ("@app:playback define stream StockStream (symbol string, price double, volume long); "
           "@info(name='q1') from StockStream[price > 60]#window.length(50) select symbol, avg(price) as a, "
           "sum(price) as s, count() as c group by symbol insert into O1; "
           "@info(name='q2') from StockStream#window.time(200 millisecond) select symbol, sum(volume) as v, "
           "count() as c group by symbol insert all events into O2;")
    check(app, [("StockStream", stock(30_000, 40, 0.1, seed=5, nulls=True)),
                ("StockStream", stock(20_000, 40, 0.1, seed=6, call=333))])


def test_e2e_query_on_another_stream_and_timers(hip_available):
    """A time window on a second stream: its timers fire while StockStream
    batches arrive (set_time once per batch on the fast path, per call on the
    per-call path) -- same chunks."""
    app = ("@app:playback define stream StockStream (symbol string, price double, volume long); "
           "define stream Other (k int, v float, b bool); "
           "@info(name='q1') from every e1=StockStream[price > 70] -> e2=StockStream[price > e1.price * 1.2] "
           "within 50 millisecond select e1.symbol as s, e1.price as p1, e2.price as p2 insert into A; "
           "@info(name='q2') from Other#window.time(5 millisecond) select k, v, b, count() as c "
           "insert all events into B;")
    n = 2_000
    b0 = stock(n, 10, 0.5, seed=7)
    t0 = int(b0.ts[0])
    other = rt.ColumnBatch(np.arange(t0 - 100, t0 - 100 + 64, dtype=np.int64),
                           [np.arange(64, dtype=np.int32), np.linspace(0, 1, 64).astype(np.float32),
                            (np.arange(64) % 2).astype(np.uint8)],
                           [None, (np.arange(64) % 7 == 0).astype(np.uint8), None],
                           np.array([0, 32, 64], np.int64))
    check(app, [("Other", other), ("StockStream", b0)])


def test_e2e_chained_query_keeps_per_call_path(hip_available):
    """q2 reads q1's output stream: the runtime pushes call by call (the
    reference's junction order), and a stream callback on the input sees one
    Event[] per call."""
    app = ("@app:playback define stream StockStream (symbol string, price double, volume long); "
           "@info(name='q1') from StockStream[price > 90] select symbol, price insert into Hi; "
           "@info(name='q2') from Hi#window.length(3) select symbol, sum(price) as s insert into O;")
    check(app, [("StockStream", stock(10_000, 20, 0.3, seed=9, call=500))], streams=("StockStream", "Hi"))
