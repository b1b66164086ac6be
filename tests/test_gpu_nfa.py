"""Generic per-key NFA engine (libsiddhi_hip engine 4) vs the CPU oracle:
config S4 shapes (counting sequences with e2[last], logical and/or, absent
`not ... for` with playback timers), unpartitioned and inside
`partition with`, across micro-batch splits and per-event calls.  Every
output row (values, nulls, timestamps, event types, callback chunking) must
be identical."""
import os

import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu

ENGINE_PATTERN, ENGINE_NFA = 1, 4
# `every e1 -> (e2 or|and e3)` runs on the forward-scan pattern engine
# (tests/test_gpu_logical.py); every other S4 shape on the generic NFA engine
# (tests/test_gpu_logical.py), and `every e1 -> not X for t` (unpartitioned) on
# the absent forward-scan engine (tests/test_gpu_absent.py)
EXPECT_ENGINE = {"or": ENGINE_PATTERN, "Por": ENGINE_PATTERN, "and": ENGINE_PATTERN, "Pand": ENGINE_PATTERN,
                 "not": ENGINE_PATTERN}


def split(sym, price, vol, ts, parts, call=1024):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])
            if b > a]


UNPART = [(k, wl.S4_APPS[k]) for k in ("seq", "seq14", "seqplus", "or", "and", "not", "bare")]
PART = [("P" + k, wl.S4_PART_APPS[k]) for k in ("seq", "seqplus", "or", "and", "not")]


@pytest.mark.parametrize("name,app", UNPART, ids=[c[0] for c in UNPART])
@pytest.mark.parametrize("parts", [1, 3])
def test_s4_unpartitioned_equals_oracle(hip_available, name, app, parts):
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(12000, 1000, 1.0, seed_offset=hash(name) % 1000)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == EXPECT_ENGINE.get(name, ENGINE_NFA)
    assert_same_rows(dev, ora)
    assert counters["events"] == len(ts)


@pytest.mark.parametrize("name,app", PART, ids=[c[0] for c in PART])
@pytest.mark.parametrize("parts", [1, 4])
def test_s4_partitioned_equals_oracle(hip_available, name, app, parts):
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(60000, 300, 1.0, seed_offset=hash(name) % 1000)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == EXPECT_ENGINE.get(name, ENGINE_NFA)
    if name != "Pseq":
        assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("name", ["seqplus", "or", "not"])
def test_s4_single_event_calls(hip_available, name):
    # B = 1: every InputHandler call carries one event (per-call time advance and timers)
    qp, _ = compile_single_query(wl.S4_APPS[name])
    sym, price, vol, ts = wl.stock_stream(3000, 20, 3.0, seed_offset=5)
    batches = [(0, stock_batch(sym, price, vol, ts, call_size=1))]
    assert_same_rows(run_device(qp, batches)[0], run_oracle(qp, batches))


def test_absent_timer_fires_on_set_time(hip_available):
    """`not ... for` partials complete on a playback time change alone
    (Scheduler.onTimeChange from InputHandler-less setCurrentTimestamp)."""
    from oracle_engine import OracleQueryEngine
    from parity import concat_rows
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    app = wl.S4_PART_APPS["not"]
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(4000, 40, 1.0, seed_offset=9)
    b = stock_batch(sym, price, vol, ts)
    t_end = int(ts[-1]) + 5000
    # oracle
    eng = OracleQueryEngine(qp, None)
    parts = []
    cid = 0
    offs = b.call_offsets
    from siddhi_amd.runtime import ColumnBatch
    for c in range(len(offs) - 1):
        s, e = int(offs[c]), int(offs[c + 1])
        sub = ColumnBatch(b.ts[s:e], [x[s:e] for x in b.cols], [None] * 3)
        for ch in eng.set_time(int(b.ts[e - 1])) + eng.push(0, sub):
            parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
            cid += 1
    for ch in eng.set_time(t_end):
        parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
        cid += 1
    eng.close()
    ora = concat_rows(parts)
    # device
    dq = DeviceQuery(qp.ir)
    dev_parts = []
    cols = [np.ascontiguousarray(x) for x in b.cols]
    tts = np.ascontiguousarray(b.ts, np.int64)
    dq.push_raw(0, b.n, tts.ctypes.data, [x.ctypes.data for x in cols], [0] * 3, SHD_MEM_HOST, b.call_offsets, True)
    r = dq.poll()
    if r is not None:
        dev_parts.append(r)
    n_before = sum(len(p[2]) for p in dev_parts)
    dq.set_time(t_end)
    r = dq.poll()
    if r is not None:
        dev_parts.append(r)
    dq.close()
    dev = concat_rows(dev_parts)
    assert len(dev[2]) > n_before   # the time change alone completed partials
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("caps", [{"SHD_NFA_LIST": "4"},
                                  {"SHD_NFA_LIST": "2", "SHD_NFA_PARTIALS": "8", "SHD_NFA_EVENTS": "8",
                                   "SHD_NFA_RECORDS": "8"}],
                         ids=["lists", "lists-pools"])
@pytest.mark.parametrize("shape", ["and", "seqplus-part"])
def test_capacity_overflow_grows(hip_available, monkeypatch, caps, shape):
    """A push whose keys outgrow the per-key lists / pools is rerun from the
    pre-push state with the overflowed capacities doubled (grow,
    never drop, never fail): started far too small, the rows still equal the
    oracle's, over several pushes (the grown layout carries on) and a snapshot
    taken after growth restores into a fresh query."""
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    for k, v in caps.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SHD_NO_LOGICAL_SCAN", "1")   # the generic engine's pending lists
    app = wl.S4_APPS["and"] if shape == "and" else wl.S4_PART_APPS["seqplus"]
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(8000, 40 if shape != "and" else 1000, 1.0, seed_offset=2)
    batches = split(sym, price, vol, ts, 3, call=500)
    ora = run_oracle(qp, batches)
    assert len(ora[2]) > 0
    dq = DeviceQuery(qp.ir)
    dev_parts = []
    try:
        for j, (si, b) in enumerate(batches):
            if j == 2:   # restore the grown state into a fresh query
                image = dq.snapshot()
                dq.close()
                dq = DeviceQuery(qp.ir)
                dq.restore(image)
            cols = [np.ascontiguousarray(x) for x in b.cols]
            tts = np.ascontiguousarray(b.ts, np.int64)
            dq.push_raw(si, b.n, tts.ctypes.data, [x.ctypes.data for x in cols], [0] * 3, SHD_MEM_HOST,
                        b.call_offsets, True)
            r = dq.poll()
            if r is not None:
                dev_parts.append(r)
    finally:
        dq.close()
    assert_same_rows(concat_rows(dev_parts), ora)


@pytest.mark.parametrize("name", ["seqplus", "not100"])
def test_window_lane_hash_collision_is_caught(hip_available, monkeypatch, name):
    """Debug hook SHD_NFA_HASH1_ZERO: the first of the two window-lane state
    hashes collides for every lane, so a wrong warm-up state would pass it;
    the second hash still rejects it (the push reruns with longer warm-ups)
    and the rows equal the oracle's."""
    monkeypatch.setenv("SHD_NFA_HASH1_ZERO", "1")
    monkeypatch.setenv("SHD_NFA_CHUNK", "5")
    monkeypatch.setenv("SHD_NO_ABSENT_SCAN", "1")
    qp, _ = compile_single_query(WINDOW_SEQS[name] if name in WINDOW_SEQS else wl.S4_APPS[name])
    sym, price, vol, ts = wl.stock_stream(20000, 50, 1.0, seed_offset=78)
    batches = split(sym, price, vol, ts, 2, call=700)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == ENGINE_NFA
    assert_same_rows(dev, ora)


WINDOW_SEQS = {
    # config S4's sequence (no match on random prices: a count below its minimum
    # does not survive resetAndUpdate) and bounded shapes that do match
    "seq": wl.S4_APPS["seq"],
    "seq13": wl.S4_APPS["seq"].replace("<2:5>", "<1:3>"),
    "seq14": wl.S4_APPS["seq"].replace("<2:5>", "<1:4>").replace("price<e2[last].price", "price<e1.price"),
    "bare": wl.S4_APPS["bare"],
    # unbounded count (`+`): the warm-up is learned (verification doubles it)
    "seqplus": wl.S4_APPS["seqplus"],
    # patterns bounded by an absent `for` time: timers fire inside the lanes
    "not": wl.S4_APPS["not"],
    "not100": wl.S4_APPS["not"].replace("price>98", "price>95").replace("for 1 sec", "for 100 milliseconds"),
}


@pytest.mark.parametrize("name", list(WINDOW_SEQS))
@pytest.mark.parametrize("chunk", ["auto", "1", "5", "64"])
@pytest.mark.parametrize("parts", [1, 4])
def test_sequence_window_lanes(hip_available, monkeypatch, name, chunk, parts):
    """Unpartitioned every-started sequences and time-bounded patterns run as
    window lanes (one lane per chunk of events; the first lanes continue the
    carried state exactly, the others replay a warm-up from a fresh state and
    are verified against their predecessor's end state; a failed check reruns
    the push with longer warm-ups): rows identical to the oracle and to the
    one-lane NFA, for lanes of one event and micro-batch cuts inside partials.
    `bare` (no every) stays on one lane."""
    if chunk != "auto":
        monkeypatch.setenv("SHD_NFA_CHUNK", chunk)
    monkeypatch.setenv("SHD_NO_ABSENT_SCAN", "1")   # `not ... for`: the NFA's window lanes, not the absent scan
    qp, _ = compile_single_query(WINDOW_SEQS[name])
    sym, price, vol, ts = wl.stock_stream(20000, 50, 1.0, seed_offset=77)
    batches = split(sym, price, vol, ts, parts, call=700)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == ENGINE_NFA
    assert_same_rows(dev, ora)
    monkeypatch.setenv("SHD_NFA_WINDOW", "0")
    one, _, _ = run_device(qp, batches)
    assert_same_rows(dev, one)
    if name in ("seq13", "seq14", "seqplus"):
        assert len(ora[2]) > 1000
    if name in ("not", "not100"):
        assert len(ora[2]) > 20
        monkeypatch.delenv("SHD_NO_ABSENT_SCAN")
        monkeypatch.delenv("SHD_NFA_WINDOW")
        scan, _, skind = run_device(qp, batches)   # the absent forward-scan engine
        assert skind == ENGINE_PATTERN
        assert_same_rows(scan, ora)
