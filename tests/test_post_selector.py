"""Selectors that aggregate or filter (`having`) over pattern / sequence
output, on the CPU.

The reference hands every StateEvent to QuerySelector as a chunk of its own
(StateMultiProcessStreamReceiver.processAndClear, C/query/input/
StateMultiProcessStreamReceiver.java:47-68; SingleProcessStreamReceiver.java:
48-72), so processInBatchNoGroupBy / processInBatchGroupBy
(C/query/selector/QuerySelector.java:271-373) emit each match whose `having`
holds, with the aggregators folded over all earlier matches.  The oracle
restates that directly on StateEvents.  libsiddhi_hip instead runs the state
plan with the selector's base values as outputs and then the selector as a
single-stream plan over those rows, one InputHandler call per row (the IR's
POST section, include/siddhi_ir.h).  Here that decomposition is checked on
the oracle itself: state plan with base outputs -> single plan over its rows
== the direct restatement, row for row."""
import copy

import numpy as np
import pytest

from oracle_engine import OracleQueryEngine
from parity import compile_single_query, run_oracle, stock_batch
from siddhi_amd import planner as pl
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

DEF = "@app:playback " + wl.STOCK_DEF + " "

APPS = [
    ("count-sum-avg", DEF + "from every e1=StockStream[price>70] -> e2=StockStream[symbol==e1.symbol and "
     "price>e1.price] within 1 sec select e1.symbol as s, count() as c, sum(e2.price) as t, "
     "avg(e1.price) as a insert into O;"),
    ("group-by", DEF + "from every e1=StockStream[price>70] -> e2=StockStream[symbol==e1.symbol] within 1 sec "
     "select e1.symbol as s, count() as c, sum(e2.volume) as v group by e1.symbol insert into O;"),
    ("having-agg", DEF + "from every e1=StockStream[price>60] -> e2=StockStream[symbol==e1.symbol and "
     "price>e1.price] within 1 sec select e2.price - e1.price as d, count() as c "
     "having c % 3 == 0 or d > 5.0 insert into O;"),
    ("having-plain-partitioned", DEF + "partition with (symbol of StockStream) begin "
     "from every e1=StockStream[price>70] -> e2=StockStream[price>e1.price] within 1 sec "
     "select e1.symbol as s, e1.price as p1, e2.price as p2 having p2 > p1 * 1.1 insert into O; end;"),
    ("sequence-count-state", DEF + "from every e1=StockStream, e2=StockStream[price>e1.price]+, "
     "e3=StockStream[price<e2[last].price] select e1.price as p, count() as c, avg(e3.price) as a "
     "having c > 1 insert into O;"),
    ("group-by-having-sum-long", DEF + "from every e1=StockStream[price>80] -> e2=StockStream[price<e1.price] "
     "within 50 milliseconds select e1.symbol as s, sum(e1.volume) as v, count() as c group by e2.symbol "
     "having v > 2000 insert into O;"),
]


def stream_batches(n, keys, dt, seed, pushes=3):
    sym, price, vol, ts = wl.stock_stream(n, keys, dt, seed_offset=seed)
    cut = np.linspace(0, n, pushes + 1).astype(int)
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call_size=97))
            for a, b in zip(cut[:-1], cut[1:])]


def _plan_a(qp):
    """The state plan with the selector's base values as outputs (what the
    device's state engine runs)."""
    base, _ = qp.plan.post
    pa = copy.deepcopy(qp.plan)
    pa.outputs = [("_b%d" % k, t, e) for k, (t, e) in enumerate(base)]
    pa.aggs, pa.group_by, pa.having, pa.post = [], [], -1, None
    return pl.QueryPlan(pa, pa.to_bytes(), qp.input_streams, [o[0] for o in pa.outputs],
                        [o[1] for o in pa.outputs], qp.target, qp.name, qp.partitioned, qp.receiver_kind)


def _plan_b(qp):
    _, sub = qp.plan.post
    return pl.QueryPlan(sub, sub.to_bytes(), ["_post"], qp.output_names, qp.output_types, qp.target, qp.name,
                        False, {"_post": "single"})


def run_decomposed(qp, batches):
    """Oracle state plan with base outputs, its rows pushed one call per row
    into an oracle running the nested single plan; chunk ids of the state
    rows are kept."""
    rows_a = run_oracle(_plan_a(qp), batches)
    chunk, typ, ts, vals, nul = rows_a
    n = len(ts)
    types = qp.plan.post[1].stream_types[0]
    eng = OracleQueryEngine(_plan_b(qp), None)
    out = []
    for i in range(n):
        cols = []
        for k, t in enumerate(types):
            b = vals[i:i + 1, k]
            if t == pl.T_INT:
                cols.append(b.astype(np.uint32).view(np.int32))
            elif t == pl.T_LONG:
                cols.append(b.view(np.int64))
            elif t == pl.T_FLOAT:
                cols.append(b.astype(np.uint32).view(np.float32))
            elif t == pl.T_DOUBLE:
                cols.append(b.view(np.float64))
            elif t == pl.T_BOOL:
                cols.append(b.astype(np.uint8))
            else:
                cols.append(b.astype(np.uint32))
        nuls = [nul[i:i + 1, k].astype(np.uint8) for k in range(len(types))]
        for ch in eng.push(0, ColumnBatch(ts[i:i + 1], cols, nuls)):
            for r in range(len(ch.ts)):
                out.append((chunk[i], ch.types[r], ch.ts[r], ch.values[r], ch.nulls[r]))
    eng.close()
    if not out:
        return None
    return (np.array([o[0] for o in out]), np.array([o[1] for o in out]), np.array([o[2] for o in out]),
            np.stack([o[3] for o in out]), np.stack([o[4] for o in out]))


@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
def test_decomposition_equals_direct_selector(name, app):
    qp, d = compile_single_query(app)
    wl.register_symbols(d, 50)
    assert qp.plan.post is not None
    batches = stream_batches(6000, 50, 0.5, seed=31)
    direct = run_oracle(qp, batches)
    dec = run_decomposed(qp, batches)
    assert len(direct[2]) > 0, "no rows: the case checks nothing"
    assert dec is not None and len(dec[2]) == len(direct[2])
    np.testing.assert_array_equal(dec[2], direct[2])
    np.testing.assert_array_equal(dec[3], direct[3])
    np.testing.assert_array_equal(dec[4], direct[4])
    # the state chunks are the callback chunks: same boundaries
    b1 = np.r_[True, dec[0][1:] != dec[0][:-1]]
    b2 = np.r_[True, direct[0][1:] != direct[0][:-1]]
    np.testing.assert_array_equal(b1, b2)


def test_count_over_pattern_counts_every_match():
    qp, d = compile_single_query(APPS[0][1])
    wl.register_symbols(d, 50)
    rows = run_oracle(qp, stream_batches(6000, 50, 0.5, seed=32))
    c = rows[3][:, 1].view(np.int64)
    np.testing.assert_array_equal(c, np.arange(1, len(c) + 1))


def test_partitioned_aggregation_is_refused():
    app = DEF + ("partition with (symbol of StockStream) begin from every e1=StockStream[price>70] -> "
                 "e2=StockStream[price>e1.price] select count() as c insert into O; end;")
    with pytest.raises(pl.UnsupportedPlanException):
        compile_single_query(app)


def test_aggregating_patterns_are_not_shared():
    from siddhi_amd import query_compiler as qc
    q = qc.parse(APPS[0][1]).execution_order[0]
    assert pl.share_signature(q) is None
