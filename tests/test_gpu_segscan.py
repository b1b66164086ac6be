"""Segmented-scan window aggregates (the default device mode for count(),
sum(double|float) and avg(numeric); engine_single.hip k_seg_*): every output
row equal to the CPU oracle's (the reference's sequential add/remove fold,
SumAttributeAggregatorExecutor.java:184-198, AvgAttributeAggregatorExecutor.java:148-166)
with doubles within 1e-9 relative and everything else -- counts, keys,
timestamps, nulls, callback boundaries -- exact.

Shapes chosen against the scan's edge cases: one group (segments spanning
many tiles, long (group, call) runs), many sparse groups, windows of length 1,
short time windows expiring most items inside a push, null arguments, no
group-by, many micro-batches (carried window items), and a switch between
the scan and the exact fold mid-stream (the group tables both modes keep)."""
import numpy as np
import pytest

from parity import assert_rows_agg, compile_single_query, concat_rows, float_cols, run_device, run_oracle
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

SCHEMA = "define stream S (k int, i int, l long, f float, d double); "

APPS = [
    ("one-group-length", "from S#window.length(5000) select k, sum(d) as s, avg(d) as a, count() as c "
                         "insert into O;"),
    ("one-group-groupby", "from S#window.length(3000) select k, sum(d) as s, avg(d) as a, count() as c "
                          "group by k insert into O;"),
    ("sparse-groups", "from S#window.time(30 milliseconds) select k, avg(d) as a, sum(d) as s, count() as c "
                      "group by k insert into O;"),
    ("length-1", "from S#window.length(1) select k, sum(d) as s, avg(d) as a, count() as c group by k "
                 "insert into O;"),
    ("time-short", "from S#window.time(2 milliseconds) select k, avg(d) as a, count() as c group by k "
                   "insert into O;"),
    ("typed-channels", "from S[d > 10.0]#window.length(400) select k, sum(f) as sf, avg(i) as ai, avg(l) as al, "
                       "sum(d) as sd, count() as c group by k insert into O;"),
]


def make_batches(seed, nbatch, m, keys, nulls=True, call=300, one_call=False):
    rng = np.random.default_rng(seed)
    out = []
    t = 50_000
    for _ in range(nbatch):
        k = rng.integers(0, keys, m).astype(np.int32)
        i = rng.integers(-1000, 1000, m).astype(np.int32)
        lv = rng.integers(-10 ** 9, 10 ** 9, m).astype(np.int64)
        f = rng.uniform(-50, 50, m).astype(np.float32)
        d = rng.uniform(0, 100, m)
        nl = [None] + [(rng.random(m) < 0.05).astype(np.uint8) if nulls else None for _ in range(4)]
        ts = t + np.sort(rng.integers(0, 4000, m)).astype(np.int64)
        t = int(ts[-1])
        offs = np.array([0, m], np.int64) if one_call else np.arange(0, m + 1, call, dtype=np.int64)
        if offs[-1] != m:
            offs = np.append(offs, m)
        out.append((0, ColumnBatch(ts, [k, i, lv, f, d], nl, offs)))
    return out


@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
@pytest.mark.parametrize("keys", [1, 7, 5000])
def test_segscan_equals_oracle(hip_available, name, app, keys):
    qp, _ = compile_single_query("@app:playback " + SCHEMA + app)
    batches = make_batches(11 + keys, 5, 20_000, keys)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == 2 and len(ora[2]) > 0
    assert_rows_agg(dev, ora, qp, exact=False)


def test_segscan_one_call_per_push(hip_available):
    """Each push is one InputHandler call: (group, call) runs as long as the
    group's share of the push (run-start search over tens of thousands)."""
    qp, _ = compile_single_query("@app:playback " + SCHEMA + APPS[1][1])
    batches = make_batches(5, 3, 60_000, 2, one_call=True)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)


def test_segscan_many_pushes_no_nulls(hip_available):
    qp, _ = compile_single_query("@app:playback " + SCHEMA + APPS[2][1])
    batches = make_batches(9, 12, 4_000, 300, nulls=False)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)


@pytest.mark.parametrize("first", ["scan", "exact"])
def test_mode_switch_midstream(hip_available, first):
    """shd_set_option("exact_aggregates") between pushes: both modes keep the
    per-group tables (window state after each push) current, so the other mode
    continues from them."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, _ = compile_single_query("@app:playback " + SCHEMA + APPS[5][1])
    batches = make_batches(21, 6, 10_000, 9)
    ora = run_oracle(qp, batches)
    dq = DeviceQuery(qp.ir)
    parts = []
    try:
        for j, (si, b) in enumerate(batches):
            exact = (j < 3) == (first == "exact")
            dq.set_option("exact_aggregates", int(exact))
            cols = [np.ascontiguousarray(c) for c in b.cols]
            nul = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in b.nulls]
            ts = np.ascontiguousarray(b.ts, np.int64)
            dq.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols],
                        [0 if x is None else x.ctypes.data for x in nul], SHD_MEM_HOST, b.call_offsets, True)
            r = dq.poll()
            if r is not None:
                parts.append(r)
    finally:
        dq.close()
    assert_rows_agg(concat_rows(parts), ora, qp, exact=False)


def test_unknown_option_rejected(hip_available):
    from siddhi_amd.hip_engine import DeviceQuery, SiddhiHipError, SHD_E_ARG
    qp, _ = compile_single_query(SCHEMA + APPS[0][1])
    dq = DeviceQuery(qp.ir)
    try:
        with pytest.raises(SiddhiHipError) as ei:
            dq.set_option("no_such_option", 1)
        assert ei.value.code == SHD_E_ARG
    finally:
        dq.close()


@pytest.mark.parametrize("shape", ["nonfinite", "wide-range", "late-inf"])
def test_range_guard_falls_back_to_exact_fold(hip_available, shape):
    """the reference's running sum stays Inf / NaN once a non-finite
    value passed (Inf - Inf), and over a wide magnitude range its rounding
    history shows (1e20 + 1 - 1e20 = 0).  The device sees such operands in a
    push and keeps the exact sequential fold from that push on: rows equal the
    oracle (NaN == NaN, Inf == Inf; within 1e-9 before the switch)."""
    qp, _ = compile_single_query("@app:playback " + SCHEMA + APPS[1][1])
    batches = make_batches(77, 5, 6_000, 5)
    rng = np.random.default_rng(3)
    for j, (_, b) in enumerate(batches):
        d = b.cols[4]
        if shape == "nonfinite" and j == 0 or shape == "late-inf" and j == 3:
            idx = rng.choice(len(d), 6, replace=False)
            d[idx[:2]] = np.inf
            d[idx[2:4]] = -np.inf
            d[idx[4:]] = np.nan
        elif shape == "wide-range":
            big = rng.random(len(d)) < 0.01
            d[big] = 1e20 * np.sign(rng.random(big.sum()) - 0.5)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)
    if shape != "late-inf":
        # exact from the first push on (NaN payload bits differ between the
        # host and the device; Java prints every NaN alike)
        def canon(rows):
            v = rows[3].copy()
            for k in float_cols(qp):
                col = v[:, k].view(np.float64)
                col[np.isnan(col)] = np.nan
            return rows[:3] + (v,) + rows[4:]
        assert_rows_agg(canon(dev), canon(ora), qp, exact=True)


def test_range_guard_spans_pushes(hip_available):
    """one length window holds items of several pushes, each push
    narrow in magnitude on its own (~1, then 1e20, then ~1 again).  The guard
    keeps the operand span over every push since reset, so the 1e20 push
    switches the query to the exact fold before the reference's running sum
    picks up the big values; when they leave the window the device's sums
    carry the same rounding residue as the reference's (1e20 + x - 1e20 != x).
    A per-push span would stay on the scans and report the exact small sums.

    (A wide magnitude range that arrives in the SAME order the other way round
    -- big values first, small ones after the scans ran -- is catastrophic
    cancellation of the reference's own history, which no reassociated scan can
    reproduce: exact_aggregates=1 is the bit-exact mode for such streams,
    include/siddhi_hip.h shd_set_option.)"""
    qp, _ = compile_single_query("@app:playback " + SCHEMA +
                                 "from S#window.length(4000) select k, sum(d) as s, count() as c insert into O;")
    batches = make_batches(91, 4, 3_000, 1, nulls=False)
    batches[1][1].cols[4][:] = 1e20 + np.arange(3_000) * 1e6
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)


CHUNK_APPS = [a for a in APPS if a[0] in ("sparse-groups", "length-1", "time-short", "typed-channels",
                                           "one-group-groupby")] + [
    ("w2-length-shape", "from S[d > 20.0]#window.length(700) select k, avg(d) as a, sum(d) as s, count() as c "
                        "group by k insert into O;"),
    ("long-window", "from S#window.length(9000) select k, sum(d) as s, count() as c group by k insert into O;"),
]


@pytest.mark.parametrize("name,app", CHUNK_APPS, ids=[a[0] for a in CHUNK_APPS])
@pytest.mark.parametrize("keys", [64, 700, 2000])
@pytest.mark.parametrize("call", [1, 97, 1024])
def test_chunked_window_walk(hip_available, monkeypatch, name, app, keys, call):
    """Dense group ids in [64, 2048]: the chunked window walk (opt-in, k_wc_*: per-chunk
    group sort in LDS, chunk-start states from a prefix over chunks, carried
    items in their own chunks) against the oracle at rtol 1e-9, and against
    the segmented scans (SHD_NO_WCHUNK) -- calls of one event, of 97 and of
    1024, windows longer than a chunk, null operands, typed channels."""
    monkeypatch.setenv("SHD_WCHUNK", "1")   # the chunked walk is opt-in
    qp, _ = compile_single_query("@app:playback " + SCHEMA + "@info(name='q') " + app)
    m = 3000 if call == 1 else 20000
    batches = make_batches(23 + keys, 4, m, keys, call=call)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == 2 and len(ora[2]) > 0
    assert_rows_agg(dev, ora, qp, exact=False)
    monkeypatch.setenv("SHD_NO_WCHUNK", "1")
    seg, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, seg, qp, exact=False)


@pytest.mark.parametrize("late", [False, True])
def test_range_guard_sign_channel(hip_available, late):
    """a window whose operands have both signs can cancel to
    far below them (+-1e8 pairs whose windows sum to a few units), where the
    reference's running `sum += v; sum -= v` keeps the rounding history of the
    big operands (SumAttributeAggregatorExecutor.java:184-198) and a
    difference of prefix sums cannot agree within 1e-9.  The guard's sign
    channel sees both signs and keeps the exact fold from that push on (late:
    the first pushes are one-signed and run on the scans)."""
    qp, _ = compile_single_query("@app:playback " + SCHEMA +
                                 "from S#window.length(64) select k, sum(d) as s, avg(d) as a, count() as c "
                                 "group by k insert into O;")
    batches = make_batches(5, 4, 8_000, 1, nulls=False)   # one group: its window alternates signs
    rng = np.random.default_rng(9)
    for j, (_, b) in enumerate(batches):
        d = b.cols[4]
        if late and j < 2:
            continue
        sign = np.where(np.arange(len(d)) % 2 == 0, 1.0, -1.0)
        d[:] = sign * 1e8 + rng.random(len(d))
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    s = ora[3][:, 1].view(np.float64)
    assert np.median(np.abs(s[len(s) // 2:])) < 1e3   # the windows do cancel
    assert_rows_agg(dev, ora, qp, exact=False)
