"""`every e1=A[f1] -> (e2=B[f2] or|and e3=B[f3]) [within W]` on the forward-scan
pattern engine (engine 1) vs the CPU oracle, and vs the generic NFA engine
(engine 4, forced with SHD_NO_LOGICAL_SCAN) on the same device.

Reference: LogicalPreStateProcessor.java:113-154 / LogicalPostStateProcessor.java:59-86
(OR: the first operand whose filter passes fills its slot, the partner slot
stays empty), MultiProcessStreamReceiver (processors in reverse setup order,
one callback chunk per (event, processor)), StateInputStreamParser.java:349-361.
Overlapping filters pin which operand wins when both pass on one event.
AND: both operands fill at their first passing event (possibly the same one);
half-filled partials carry their operand event across pushes."""
import zlib

import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

ENGINE_PATTERN, ENGINE_NFA = 1, 4
HEAD = "@app:playback " + wl.STOCK_DEF + " "


def split(sym, price, vol, ts, parts, call=1024):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])
            if b > a]


def q(second, within="", sel="e1.price as p1, e2.price as p2, e3.price as p3"):
    return ("@info(name='q') from every e1=StockStream[price>70] -> " + second + within +
            " select " + sel + " insert into O;")


OR_CASES = [
    ("s4-or", HEAD + q("(e2=StockStream[price>e1.price] or e3=StockStream[price<e1.price*0.9])")),
    # both operands often pass on the same event: the first operand wins
    ("overlap-first", HEAD + q("(e2=StockStream[price>e1.price] or e3=StockStream[price>e1.price*0.99])")),
    ("overlap-second", HEAD + q("(e2=StockStream[price>e1.price*0.99] or e3=StockStream[price>e1.price])")),
    ("within", HEAD + q("(e2=StockStream[price>e1.price*1.2] or e3=StockStream[price<e1.price*0.75])",
                        " within 6 milliseconds")),
    ("partitioned", HEAD + "partition with (symbol of StockStream) begin " +
     q("(e2=StockStream[price>e1.price] or e3=StockStream[price<e1.price*0.9])", " within 1 sec",
       "e1.symbol as s, e1.price as p1, e2.price as p2, e3.price as p3") + " end;"),
    ("ts-output", HEAD + q("(e2=StockStream[price>e1.price*1.1] or e3=StockStream[price<e1.price*0.8])", "",
                           "e1.price as p1, e2.price as p2, e3.price as p3, eventTimestamp() as t")),
    # the plain two-state form through the same projection: eventTimestamp() of a
    # match is the completing event's (StreamPostStateProcessor.java:64-83)
    ("p1-ts-output", HEAD + "@info(name='q') from every e1=StockStream[price>70] -> "
     "e2=StockStream[price>e1.price and eventTimestamp() - e1.price > 0] "
     "select e1.price as p1, e2.price as p2, eventTimestamp() as t insert into O;"),
]


AND_CASES = [
    ("s4-and", wl.S4_APPS["and"]),
    # one event often passes both operands: it fills both and completes at once
    ("and-overlap", HEAD + q("e2=StockStream[price>e1.price] and e3=StockStream[price>e1.price*1.01]",
                             " within 20 milliseconds")),
    # the first operand's filter reads the partner's slot (null until filled; the
    # parser compiles the second operand first, so only this direction resolves)
    ("and-partner-ref", HEAD + q("e2=StockStream[price>e1.price and not (e3.price is null)] and "
                                 "e3=StockStream[price<e1.price*0.95]", " within 30 milliseconds")),
    ("and-long-carry", HEAD + q("e2=StockStream[price>e1.price*1.3] and e3=StockStream[price<e1.price*0.75]",
                                " within 3 sec")),
    ("and-partitioned", HEAD + "partition with (symbol of StockStream) begin " +
     q("e2=StockStream[price>e1.price*1.1] and e3=StockStream[price<e1.price*0.9]", " within 1 sec",
       "e1.symbol as s, e1.price as p1, e2.price as p2, e3.price as p3, eventTimestamp() as t") + " end;"),
]


@pytest.mark.parametrize("name,app", AND_CASES, ids=[c[0] for c in AND_CASES])
@pytest.mark.parametrize("parts", [1, 5])
def test_logical_and_equals_oracle(hip_available, name, app, parts):
    qp, _ = compile_single_query(app)
    keys = 40 if name == "and-partitioned" else 1000
    sym, price, vol, ts = wl.stock_stream(20000, keys, 1.0, seed_offset=zlib.crc32(name.encode()) % 1000)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("name,app", AND_CASES[:3], ids=[c[0] for c in AND_CASES[:3]])
def test_logical_and_scan_equals_generic_nfa(hip_available, monkeypatch, name, app):
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(30000, 1000, 1.0, seed_offset=17)
    batches = split(sym, price, vol, ts, 4)
    scan, _, k1 = run_device(qp, batches)
    monkeypatch.setenv("SHD_NO_LOGICAL_SCAN", "1")
    nfa, _, k2 = run_device(qp, batches)
    assert (k1, k2) == (ENGINE_PATTERN, ENGINE_NFA)
    assert_same_rows(scan, nfa)


def test_logical_and_single_event_calls(hip_available):
    qp, _ = compile_single_query(AND_CASES[1][1])
    sym, price, vol, ts = wl.stock_stream(3000, 20, 3.0, seed_offset=13)
    batches = [(0, stock_batch(sym, price, vol, ts, call_size=1))]
    assert_same_rows(run_device(qp, batches)[0], run_oracle(qp, batches))


@pytest.mark.parametrize("name,app", OR_CASES, ids=[c[0] for c in OR_CASES])
@pytest.mark.parametrize("parts", [1, 4])
def test_logical_or_equals_oracle(hip_available, name, app, parts):
    qp, _ = compile_single_query(app)
    keys = 40 if name == "partitioned" else 1000
    sym, price, vol, ts = wl.stock_stream(20000, keys, 1.0, seed_offset=zlib.crc32(name.encode()) % 1000)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["events"] == len(ts)


@pytest.mark.parametrize("name,app", OR_CASES[:3], ids=[c[0] for c in OR_CASES[:3]])
def test_logical_or_scan_equals_generic_nfa(hip_available, monkeypatch, name, app):
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(30000, 1000, 1.0, seed_offset=7)
    batches = split(sym, price, vol, ts, 3)
    scan, _, k1 = run_device(qp, batches)
    monkeypatch.setenv("SHD_NO_LOGICAL_SCAN", "1")
    nfa, _, k2 = run_device(qp, batches)
    assert (k1, k2) == (ENGINE_PATTERN, ENGINE_NFA)
    assert_same_rows(scan, nfa)


def test_logical_or_single_event_calls(hip_available):
    qp, _ = compile_single_query(OR_CASES[1][1])
    sym, price, vol, ts = wl.stock_stream(3000, 20, 3.0, seed_offset=11)
    batches = [(0, stock_batch(sym, price, vol, ts, call_size=1))]
    assert_same_rows(run_device(qp, batches)[0], run_oracle(qp, batches))


@pytest.mark.parametrize("op", ["or", "and"])
def test_logical_two_streams(hip_available, op):
    """e1 on A, both operands on B: B has two processors, so every B event
    with matches gives one chunk per operand (MultiProcessStreamReceiver)."""
    app = ("define stream A (k int, p double); define stream B (k int, p double); "
           "@info(name='q') from every e1=A[p>20] -> (e2=B[p>e1.p] %s e3=B[p<e1.p*0.5]) within 40 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2, e3.p as p3 insert into O;" % op)
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(9)
    batches = []
    t = 1000
    for r in range(40):
        si = int(rng.integers(0, 2))
        m = int(rng.integers(1, 300))
        k = rng.integers(0, 30, m).astype(np.int32)
        p = rng.uniform(0, 100, m)
        ts = t + np.sort(rng.integers(0, 20, m)).astype(np.int64)
        t = int(ts[-1])
        batches.append((si, ColumnBatch(ts, [k, p], [None, None], np.array([0, m], np.int64))))
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


MODE_CASES = [
    ("p1", wl.P1_APP, 30000, 1000, 1.0),
    ("p1-dense", wl.P1_APP, 30000, 50, 0.2),
    ("p3-dense", wl.P3_APP, 100000, 2000, 0.05),
    ("or-within", OR_CASES[3][1], 20000, 1000, 1.0),
    ("or-overlap", OR_CASES[1][1], 20000, 1000, 1.0),
    ("or-partitioned", OR_CASES[4][1], 20000, 40, 1.0),
    # ~1000 same-key events per `within` span: walks beyond the 64-position cap
    ("p1-long", wl.P1_APP, 40000, 20, 0.05),
    ("or-part-long", OR_CASES[4][1], 40000, 20, 0.05),
    # AND: wave-cooperative walks keep the operand state between 64-position
    # rounds (mode 3 is not offered for AND and falls back to the default)
    ("and-s4", AND_CASES[0][1], 20000, 1000, 1.0),
    ("and-overlap", AND_CASES[1][1], 20000, 1000, 1.0),
    ("and-partner-ref", AND_CASES[2][1], 20000, 1000, 1.0),
    ("and-long-carry", AND_CASES[3][1], 30000, 1000, 0.5),
    ("and-part-long", AND_CASES[4][1], 40000, 20, 0.05),
]


@pytest.mark.parametrize("mode", ["0", "1", "2", "3"])
@pytest.mark.parametrize("name,app,n,keys,delta", MODE_CASES, ids=[c[0] for c in MODE_CASES])
def test_resume_modes_equal_oracle(hip_available, monkeypatch, mode, name, app, n, keys, delta):
    """Deferred walks: 16 positions per thread (0), one lane per partial (1),
    one wave per partial with ballots over 64 positions (2), lane walks capped
    at 64 positions continued one wave per partial (3) -- same outputs."""
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=zlib.crc32(name.encode()) % 1000)
    batches = split(sym, price, vol, ts, 3)
    ora = run_oracle(qp, batches)
    monkeypatch.setenv("SHD_RESUME_MODE", mode)
    monkeypatch.setenv("SHD_BPOS", "1")   # position-major e2 attributes whenever walks are dense
    dev, counters, kind = run_device(qp, batches)
    assert kind == ENGINE_PATTERN
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
