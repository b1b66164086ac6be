"""Runs a known-answer case (tests/golden/kat/*.json) through the host API
(SiddhiManager -> SiddhiAppRuntime -> InputHandler -> callbacks) with a given
query-engine factory, and checks the reference test's expectations.
"""
import glob
import json
import os

import numpy as np

from siddhi_amd import runtime as rt

KAT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat")


def load_cases():
    cases = []
    for f in sorted(glob.glob(os.path.join(KAT_DIR, "*.json"))):
        with open(f) as fp:
            cases.extend(json.load(fp))
    return cases


def _py(v):
    if isinstance(v, dict):
        (k, x), = v.items()
        if k == "float":
            return ("f", float(np.float32(x)))
        return ("n", x)
    return ("v", v)


def values_equal(expected, actual, rtol=0.0):
    """rtol: relative tolerance for double results (the device's default
    segmented-scan window aggregates, BASELINE.json: within 1e-9 relative)."""
    kind, e = _py(expected)
    if e is None or actual is None:
        return e is None and actual is None
    if isinstance(e, str) or isinstance(actual, str) or isinstance(e, bool) or isinstance(actual, bool):
        return e == actual
    if kind == "f":
        return float(np.float32(actual)) == e
    if float(e) == float(actual) or (isinstance(e, int) and isinstance(actual, int) and e == actual):
        return True
    return rtol > 0 and isinstance(actual, float) and abs(float(e) - actual) <= rtol * abs(float(e))


TICK_MS = 10   # granularity of the emulated wall clock during sleeps / waits


class Collector:
    def __init__(self):
        self.in_events = []
        self.remove_events = []
        self.chunks = []


def run_case(case, engine_factory):
    mgr = rt.SiddhiManager(engine_factory=engine_factory)
    app = mgr.createSiddhiAppRuntime(case["app"])
    col = Collector()
    cb = case["callback"]
    if cb["kind"] == "query":
        class QC(rt.QueryCallback):
            def receive(self, ts, inEvents, removeEvents):
                col.chunks.append((inEvents or [], removeEvents or []))
                if inEvents:
                    col.in_events.extend(inEvents)
                if removeEvents:
                    col.remove_events.extend(removeEvents)
        app.addCallback(cb["name"], QC())
    else:
        class SC(rt.StreamCallback):
            def receive(self, events):
                col.chunks.append((events, []))
                col.in_events.extend(events)
        app.addCallback(cb["name"], SC())
    handlers = {}
    # wall-clock apps: replay the recorded clock (the first step's time is the
    # clock at start(); TestUtil / Thread.sleep steps advance it)
    first = case["sends"][0]
    clock = case.get("start_time") or first.get("ts", first.get("time", 0))
    app.clock = lambda: clock
    app.start()
    def tick_to(target):
        # wall-clock time passes continuously: due timers fire (close to) on
        # time, with the app clock at their due time (Scheduler on a wall clock)
        nonlocal clock
        while clock < target:
            clock = min(target, clock + TICK_MS)
            app.advanceTime(clock)

    for s in case["sends"]:
        if "time" in s:          # Thread.sleep on a wall-clock app
            tick_to(s["time"])
            continue
        if "idle" in s:          # Thread.sleep on a playback app with idle.time (heartbeat)
            app.idle(s["idle"])
            continue
        if "wait" in s:          # TestUtil.waitForInEvents(sleep, cb, retry) (T/TestUtil.java:69-79),
            # SiddhiTestHelper.waitForEvents(sleep, until, counter, timeout) (C/util/SiddhiTestHelper.java:49-57)
            until = s.get("until")
            for _ in range(s["retry"]):
                if until is not None and len(col.in_events) >= until:
                    break
                tick_to(clock + s["wait"])
                if until is None and len(col.in_events) == 1:
                    break
            continue
        clock = max(clock, s["ts"])
        h = handlers.get(s["stream"]) or app.getInputHandler(s["stream"])
        handlers[s["stream"]] = h
        data = [_py(v)[1] for v in s["data"]]
        h.send(s["ts"], data)
    app.shutdown()
    return col


def check_case(case, col, rtol=0.0):
    errs = []
    want = case.get("expected_count")
    if want is not None and case["callback"]["kind"] == "stream" and case.get("expected_remove_count") is not None:
        # a StreamCallback receives the expired events of `insert all events` as events too
        want += case["expected_remove_count"]
    if want is not None and len(col.in_events) != want:
        errs.append("count %d != expected %d" % (len(col.in_events), want))
    if case.get("expected_remove_count") is not None and case["callback"]["kind"] == "query" \
            and len(col.remove_events) != case["expected_remove_count"]:
        errs.append("remove count %d != expected %d" % (len(col.remove_events), case["expected_remove_count"]))
    for exp in case.get("expected_rows", []):
        n = exp["n"]
        if n == "all":
            targets = col.in_events
        elif n == "first_of_each":
            targets = [c[0][0] for c in col.chunks if c[0]]
        else:
            if n - 1 >= len(col.in_events):
                if not exp.get("if_arrived"):
                    errs.append("missing event #%d" % n)
                continue
            targets = [col.in_events[n - 1]]
        for ev in targets:
            d = ev.getData()
            if len(d) != len(exp["data"]) or not all(values_equal(e, a, rtol) for e, a in zip(exp["data"], d)):
                errs.append("event %s: %r != expected %r" % (n, d, [_py(v)[1] for v in exp["data"]]))
    for cell in case.get("expected_nth", []):
        # the n-th event a counting StreamCallback sees, one column checked
        if cell["n"] - 1 >= len(col.in_events):
            errs.append("missing event #%d" % cell["n"])
            continue
        d = col.in_events[cell["n"] - 1].getData()
        if cell["col"] >= len(d) or not values_equal(cell["value"], d[cell["col"]], rtol):
            errs.append("event #%d col %d: %r != expected %r" % (cell["n"], cell["col"], d[cell["col"]] if
                                                                  cell["col"] < len(d) else None,
                                                                  _py(cell["value"])[1]))
    for k, n in case.get("expected_chunk_sizes", {}).items():
        # callbacks that received exactly k events (T/query/window/LengthBatchWindowTestCase.java)
        got = sum(1 for c in col.chunks if len(c[0]) + len(c[1]) == int(k))
        if got != n:
            errs.append("%d chunks of %s events, expected %d" % (got, k, n))
    for cell in case.get("expected_cells", []):
        targets = [c[0][0] for c in col.chunks if c[0]] if cell["which"] == "first_of_each" else col.in_events
        for ev in targets:
            d = ev.getData()
            if cell["col"] >= len(d) or d[cell["col"]] != cell["value"]:
                errs.append("cell %d of %r != %r" % (cell["col"], d, cell["value"]))
                break
    return errs
