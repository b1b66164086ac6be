"""Query groups (shd_group_*): pattern queries on one stream that differ only
in the start state's filter run one forward scan; each member's rows must
equal the CPU oracle's for that query alone, row for row and bit-exact
(values, types, timestamps, callback chunks), across pushes (carried
partials), for unpartitioned / partitioned / two-stream patterns, threshold
families (one leader bound) and mixed filters (the leader's disjunction), and
after the group dissolves into per-member NFA engines (time going back inside
a key).  Length-window group-by aggregates that differ only in the window
length share one filter pass and item buffer; each member's rows equal its own
oracle run (doubles within 1e-9 relative).

Reference: StreamJunction.sendEvent fan-out (C/stream/StreamJunction.java:146-272);
per-partial independence of `every e1 -> e2` (ST/StreamPreStateProcessor.java:118-129,326-403)."""
import numpy as np
import pytest

from parity import assert_same_rows, concat_rows, run_oracle
from siddhi_amd import planner as pl
from siddhi_amd import query_compiler as qc
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

SCHEMA = ("@app:playback define stream S (k int, p double, v long); "
          "define stream T (k int, p double, v long); ")
BODY = "within 20 milliseconds select e1.k as k, e1.p as p1, e2.p as p2, e2.v as v2 insert into O%d;"
THRESHOLDS = [40.0 + 3.5 * i for i in range(9)]
MIXED = ["p > 70", "v < 500 and p > 40", "p < 30 or v > 900", "p > 55", "v == 7"]


def threshold_app(partitioned=False, two_stream=False):
    qs = []
    for i, th in enumerate(THRESHOLDS):
        second = "T" if two_stream else "S"
        qs.append("@info(name='q%d') from every e1=S[p > %r] -> e2=%s[k == e1.k and p > e1.p * 1.02] " % (i, th, second)
                  + BODY % i)
    body = " ".join(qs)
    if partitioned:
        return SCHEMA + "partition with (k of S) begin " + body + " end;"
    return SCHEMA + body


def mixed_app():
    qs = ["@info(name='m%d') from every e1=S[%s] -> e2=S[k == e1.k and p > e1.p] " % (i, f) + BODY % i
          for i, f in enumerate(MIXED)]
    return SCHEMA + " ".join(qs)


def make_batches(seed, nbatch, m, keys, two_stream=False, back=False, call=64):
    rng = np.random.default_rng(seed)
    out = []
    t = 1_000
    for b in range(nbatch):
        k = rng.integers(0, keys, m).astype(np.int32)
        p = rng.uniform(0, 100, m)
        v = rng.integers(0, 1000, m).astype(np.int64)
        ts = t + np.cumsum(rng.choice([0, 1, 1, 2], m)).astype(np.int64)
        if back and b == 2:
            ts -= 60          # this push starts before the previous one ended
        t = int(ts.max()) + 1
        offs = np.arange(0, m + 1, call, dtype=np.int64)
        if offs[-1] != m:
            offs = np.append(offs, m)
        si = (b % 2) if two_stream else 0
        out.append((si, ColumnBatch(ts, [k, p, v], [None, None, None], offs)))
    return out


def member_plans(app_text):
    app = qc.parse(app_text)
    d = pl.StringDictionary()
    item = app.execution_order[0]
    if isinstance(item, qc.Partition):
        queries, part = item.queries, item
    else:
        queries, part = list(app.execution_order), None
    plans = [pl.plan_query(app, q, d, part) for q in queries]
    groups = pl.share_groups(queries)
    assert groups == [list(range(len(queries)))]
    leader = pl.plan_shared_leader(app, queries, d, part)
    return plans, leader


def run_group(plans, leader, batches):
    from siddhi_amd.hip_engine import DeviceGroup, DeviceQuery, SHD_MEM_HOST
    dqs = [DeviceQuery(p.ir) for p in plans]
    g = DeviceGroup(leader.ir, dqs)
    parts = [[] for _ in dqs]
    try:
        for si, b in batches:
            cols = [np.ascontiguousarray(c) for c in b.cols]
            ts = np.ascontiguousarray(b.ts, np.int64)
            g.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols], [0, 0, 0], SHD_MEM_HOST,
                       b.call_offsets, True)
            for i, dq in enumerate(dqs):
                r = dq.poll()
                if r is not None:
                    parts[i].append(r)
        kinds = [dq.engine_kind for dq in dqs]
        counters = [dq.counters() for dq in dqs]
        shared = g.counters()
    finally:
        g.close()
        for dq in dqs:
            dq.close()
    return [concat_rows(p) for p in parts], kinds, counters, shared


@pytest.mark.parametrize("shape", ["plain", "partitioned", "two-stream", "mixed"])
def test_group_members_equal_oracle(hip_available, shape):
    app = mixed_app() if shape == "mixed" else threshold_app(shape == "partitioned", shape == "two-stream")
    plans, leader = member_plans(app)
    batches = make_batches(11 + len(shape), 4, 6_000, 40, two_stream=shape == "two-stream")
    dev, kinds, counters, shared = run_group(plans, leader, batches)
    assert all(k == 1 for k in kinds)
    total = 0
    for qp, d, c in zip(plans, dev, counters):
        ora = run_oracle(qp, batches)
        assert_same_rows(d, ora)
        assert c["events"] == sum(b.n for _, b in batches)
        assert c["matches"] == len(ora[2])
        total += len(ora[2])
    assert total > 0
    assert shared["events"] == counters[0]["events"]


def test_group_dissolves_into_member_nfa_engines(hip_available):
    """A push going back in time inside a key under `within`: the leader's open
    partials are replayed into each member's generic NFA engine, which then
    takes the batch (and every later one) alone."""
    plans, leader = member_plans(threshold_app())
    batches = make_batches(5, 4, 3_000, 25, back=True)
    dev, kinds, _, _ = run_group(plans, leader, batches)
    assert all(k == 4 for k in kinds)
    for qp, d in zip(plans, dev):
        assert_same_rows(d, run_oracle(qp, batches))


def test_group_refusals(hip_available):
    from siddhi_amd.hip_engine import DeviceGroup, DeviceQuery, SiddhiHipError
    plans, leader = member_plans(threshold_app())
    dqs = [DeviceQuery(p.ir) for p in plans[:3]]
    try:
        g = DeviceGroup(leader.ir, dqs)
        with pytest.raises(SiddhiHipError):
            dqs[0].reset()
        with pytest.raises(SiddhiHipError):
            dqs[0].snapshot()
        with pytest.raises(SiddhiHipError):   # already grouped
            DeviceGroup(leader.ir, [dqs[1]])
        g.close()
        dqs[0].reset()                        # detached: plain queries again
        # a member whose f2 differs from the leader's
        other, _ = member_plans(threshold_app().replace("1.02", "1.03"))
        odd = DeviceQuery(other[0].ir)
        try:
            with pytest.raises(SiddhiHipError):
                DeviceGroup(leader.ir, [dqs[0], odd])
        finally:
            odd.close()
    finally:
        for dq in dqs:
            dq.close()


WINDOW_LENGTHS = [1, 7, 60, 300, 1000]


def window_app(lengths, alt_filter=None):
    qs = []
    for i, ln in enumerate(lengths):
        f = alt_filter if (alt_filter and i == 1) else "p > 20.0"
        qs.append("@info(name='w%d') from S[%s]#window.length(%d) select k, avg(p) as a, sum(p) as s, count() as c "
                  "group by k insert into W%d;" % (i, f, ln, i))
    return SCHEMA + " ".join(qs)


@pytest.mark.parametrize("keys", [9, 40, 2000])
def test_window_group_members_equal_oracle(hip_available, keys):
    """Length-window group-by aggregates that differ only in the window length
    share one filter pass and one item buffer (the leader holds the longest
    window); each member's rows -- one per (call, group), first-seen order --
    equal its own oracle run (doubles within 1e-9 relative, counts exact),
    across pushes and calls of 64 events.  2000 keys: the hashed call-window
    kernel; fewer: the direct-mapped one."""
    from parity import assert_rows_agg
    plans, leader = member_plans(window_app(WINDOW_LENGTHS))
    batches = make_batches(21 + keys, 4, 6_000, keys)
    dev, kinds, counters, shared = run_group(plans, leader, batches)
    assert all(k == 2 for k in kinds)
    for qp, d, c in zip(plans, dev, counters):
        ora = run_oracle(qp, batches)
        assert len(ora[2]) > 0
        assert_rows_agg(d, ora, qp, exact=False)
        assert c["matches"] == len(ora[2])
    assert shared["events"] == counters[0]["events"]


def test_window_group_refusals(hip_available):
    from siddhi_amd.hip_engine import DeviceGroup, DeviceQuery, SiddhiHipError
    plans, leader = member_plans(window_app(WINDOW_LENGTHS[:3]))
    # a member whose filter differs from the leader's
    other = [pl.plan_query(qc.parse(window_app(WINDOW_LENGTHS[:3], "p > 21.0")),
                           list(qc.parse(window_app(WINDOW_LENGTHS[:3], "p > 21.0")).execution_order)[1],
                           pl.StringDictionary())]
    dqs = [DeviceQuery(plans[0].ir), DeviceQuery(other[0].ir)]
    try:
        with pytest.raises(SiddhiHipError):
            DeviceGroup(leader.ir, dqs)
        g = DeviceGroup(leader.ir, dqs[:1])   # a plain member is fine
        g.close()
    finally:
        for dq in dqs:
            dq.close()


@pytest.mark.parametrize("trip", ["nan", "inf", "mixed-sign", "big-call"])
def test_window_group_dissolves_into_members(hip_available, trip):
    """An operand the shared segmented pass cannot take (NaN / Inf, both
    signs) or a call beyond the call-window shape: the group dissolves before
    that push -- each member adopts its window (a suffix of the leader's
    carried items) and takes that push and every later one alone (exact fold
    from the guard's trip on); every member still equals its own oracle run."""
    from parity import assert_rows_agg
    plans, leader = member_plans(window_app(WINDOW_LENGTHS))
    batches = make_batches(91, 4, 6_000, 9)
    si, b = batches[2]
    p = b.cols[1].copy()
    if trip == "nan":
        p[100] = np.nan
    elif trip == "inf":
        p[100] = np.inf
    elif trip == "mixed-sign":
        p[100:3000:7] = -p[100:3000:7]
    offs = b.call_offsets
    if trip == "big-call":
        offs = np.array([0, 2000, b.n], np.int64)   # calls above 1024 events
    batches[2] = (si, ColumnBatch(b.ts, [b.cols[0], p, b.cols[2]], b.nulls, offs))
    dev, kinds, counters, _ = run_group(plans, leader, batches)
    assert all(k == 2 for k in kinds)
    for qp, d, c in zip(plans, dev, counters):
        ora = run_oracle(qp, batches)
        assert len(ora[2]) > 0
        assert_rows_agg(d, ora, qp, exact=False)
        assert c["matches"] == len(ora[2])
