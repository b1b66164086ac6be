"""Keyed exact window engine (engine_window.hip): windows whose selector emits
EXPIRED events (`insert all events` / `insert expired events`), `having`,
and window / aggregate queries inside `partition with (...)`, each against the
CPU oracle row for row -- values, types (CURRENT / EXPIRED), timestamps
(EXPIRED rows carry the expiry time), nulls and callback-chunk boundaries,
bit-exact (the aggregator states fold sequentially in the reference's order).

Reference: LengthWindowProcessor.java:105-142, TimeWindowProcessor.java:132-169
with the Scheduler's TIMER chunks (Scheduler.java:71-104,113-209),
QuerySelector.java:161-205 / :271-313 / :315-373, PartitionStreamReceiver.java:175-216,
PartitionStateHolder.java:43-69."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

SCHEMA = "@app:playback define stream S (k int, i int, l long, f float, d double); "

APPS = [
    ("length-all-plain", "from S#window.length(50) select k, d insert all events into O;"),
    ("length-expired-agg", "from S#window.length(30) select k, sum(d) as s, count() as c "
                           "insert expired events into O;"),
    ("length-all-groupby", "from S[d > 20.0]#window.length(40) select k, avg(d) as a, count() as c group by k "
                           "insert all events into O;"),
    ("time-all-groupby", "from S#window.time(20 milliseconds) select k, sum(d) as s, count() as c group by k "
                         "insert all events into O;"),
    ("time-expired-plain", "from S#window.time(5 milliseconds) select k, d, l insert expired events into O;"),
    ("time-all-agg", "from S[i > -500]#window.time(12 milliseconds) select sum(f) as sf, avg(i) as ai, "
                     "count() as c insert all events into O;"),
    ("part-length-all", "partition with (k of S) begin from S#window.length(3) select k, sum(d) as s, count() as c "
                        "insert all events into O; end;"),
    ("part-length-current", "partition with (k of S) begin from S#window.length(4) select k, sum(l) as s, "
                            "avg(f) as a insert into O; end;"),
    ("part-time-all", "partition with (k of S) begin from S#window.time(10 milliseconds) select k, sum(d) as s "
                      "insert all events into O; end;"),
    ("part-time-expired-groupby", "partition with (k of S) begin from S#window.time(8 milliseconds) "
                                  "select k, i, count() as c group by i insert expired events into O; end;"),
    ("part-length-groupby", "partition with (k of S) begin from S[d < 80.0]#window.length(5) "
                            "select k, i, sum(d) as s group by i insert into O; end;"),
    ("part-noagg-window", "partition with (k of S) begin from S#window.length(2) select k, d "
                          "insert all events into O; end;"),
    ("part-nowindow-agg", "partition with (k of S) begin from S select k, count() as c, sum(l) as s "
                          "insert into O; end;"),
    ("nowindow-expired", "from S select k, d insert expired events into O;"),
]


def make_batches(seed, nbatch, m, keys, call=37, gap=3, nulls=True, ivals=5):
    rng = np.random.default_rng(seed)
    out = []
    t = 10_000
    for _ in range(nbatch):
        k = rng.integers(0, keys, m).astype(np.int32)
        i = rng.integers(0, ivals, m).astype(np.int32)
        lv = rng.integers(-10 ** 6, 10 ** 6, m).astype(np.int64)
        f = rng.uniform(-50, 50, m).astype(np.float32)
        d = rng.uniform(0, 100, m)
        nl = [None, None] + [(rng.random(m) < 0.05).astype(np.uint8) if nulls else None for _ in range(3)]
        # playback time: mostly increasing with repeats, some steps back, pauses
        steps = rng.choice([0, 0, 1, 1, 2, 5, -3], m)
        ts = t + np.cumsum(steps).astype(np.int64)
        ts[rng.random(m) < 0.02] += 40   # pauses: windows drain, timers fire
        t = int(ts.max()) + gap
        offs = np.arange(0, m + 1, call, dtype=np.int64)
        if offs[-1] != m:
            offs = np.append(offs, m)
        out.append((0, ColumnBatch(ts, [k, i, lv, f, d], nl, offs)))
    return out


@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
@pytest.mark.parametrize("keys", [1, 9])
def test_window_x_equals_oracle(hip_available, name, app, keys):
    qp, _ = compile_single_query(SCHEMA + app)
    batches = make_batches(7 + keys + len(name), 4, 1_500, keys)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == 2
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("name,app", [a for a in APPS if "time" in a[0]], ids=[a[0] for a in APPS if "time" in a[0]])
def test_window_x_clock_moves_between_pushes(hip_available, name, app):
    """One InputHandler call per push and shd_set_time between them (the
    runtime's path: setCurrentTimestamp fires due TIMER chunks before the call's
    events, and wall-clock ticks fire them with no events at all)."""
    from oracle_engine import OracleQueryEngine
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query(SCHEMA + app)
    batches = make_batches(31, 2, 400, 5, call=1)
    eng = OracleQueryEngine(qp, None)
    dq = DeviceQuery(qp.ir)
    ora_parts, dev_parts = [], []
    cid = 0
    try:
        for si, b in batches:
            for c in range(b.n):
                sub = ColumnBatch(b.ts[c:c + 1], [x[c:c + 1] for x in b.cols],
                                  [None if x is None else x[c:c + 1] for x in b.nulls])
                moves = [int(b.ts[c])] if c % 3 else [int(b.ts[c]) - 7, int(b.ts[c])]
                for t in moves:
                    for ch in eng.set_time(t):
                        ora_parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                        cid += 1
                    dq.set_time(t)
                    r = dq.poll()
                    if r is not None:
                        dev_parts.append(r)
                for ch in eng.push(si, sub):
                    ora_parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                    cid += 1
                cols = [np.ascontiguousarray(x) for x in sub.cols]
                nuls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in sub.nulls]
                ts = np.ascontiguousarray(sub.ts, np.int64)
                dq.push_raw(si, 1, ts.ctypes.data, [x.ctypes.data for x in cols],
                            [0 if x is None else x.ctypes.data for x in nuls], SHD_MEM_HOST, None, False)
                r = dq.poll()
                if r is not None:
                    dev_parts.append(r)
    finally:
        eng.close()
        dq.close()
    assert_same_rows(concat_rows(dev_parts), concat_rows(ora_parts))


@pytest.mark.parametrize("name,app", [a for a in APPS if a[0] in ("part-time-all", "length-all-groupby",
                                                                  "time-all-agg")],
                         ids=["part-time-all", "length-all-groupby", "time-all-agg"])
def test_window_x_snapshot_restore_midstream(hip_available, name, app):
    """shd_snapshot after two pushes, restore into a fresh query: the rest of
    the stream gives the rows of an uninterrupted run."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query(SCHEMA + app)
    batches = make_batches(55, 4, 900, 6)
    ora = run_oracle(qp, batches)

    def push(dq, si, b):
        cols = [np.ascontiguousarray(c) for c in b.cols]
        nuls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in b.nulls]
        ts = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols],
                    [0 if x is None else x.ctypes.data for x in nuls], SHD_MEM_HOST, b.call_offsets, True)
        return dq.poll()

    parts = []
    dq = DeviceQuery(qp.ir)
    for si, b in batches[:2]:
        r = push(dq, si, b)
        if r is not None:
            parts.append(r)
    image = dq.snapshot()
    dq.close()
    dq2 = DeviceQuery(qp.ir)
    try:
        dq2.restore(image)
        for si, b in batches[2:]:
            r = push(dq2, si, b)
            if r is not None:
                parts.append(r)
    finally:
        dq2.close()
    assert_same_rows(concat_rows(parts), ora)


def test_window_x_big_push_many_keys(hip_available):
    """200 k events over 20 k partition keys in three pushes (long segments,
    many TIMER chunks per clock move, carried FIFOs of every key)."""
    qp, _ = compile_single_query(SCHEMA + APPS[8][1])
    batches = make_batches(99, 3, 70_000, 20_000, call=1024)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
