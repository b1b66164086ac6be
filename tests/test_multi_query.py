"""Config M5 (BASELINE.json configs[4]): 100 pattern + window
queries sharing one StockStream junction (StreamJunction.sendEvent fan-out to
every subscribed receiver in definition order, C/stream/StreamJunction.java:146-272).

Each query's callback output (rows, timestamps, expired flags, and the
grouping of rows into callback invocations) must be identical between the
device runtime (libsiddhi_hip, one device query per query) and the CPU
oracle runtime on the same InputHandler calls.
"""
import numpy as np
import pytest

from oracle_engine import OracleQueryEngine
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch, QueryCallback, SiddhiManager


class _Rec(QueryCallback):
    def __init__(self, out):
        self.out = out

    def receive(self, timestamp, inEvents, removeEvents):
        self.out.append((timestamp,
                         [(e.getTimestamp(), tuple(e.getData())) for e in (inEvents or [])],
                         [(e.getTimestamp(), tuple(e.getData())) for e in (removeEvents or [])]))


def run_app(app, factory, n, keys, delta, seed=5, call=256):
    m = SiddhiManager(engine_factory=factory) if factory else SiddhiManager()
    rt = m.createSiddhiAppRuntime(app)
    wl.register_symbols(rt.dictionary, keys)
    outs = {}
    for q in rt.queries:
        outs[q.name] = []
        rt.addCallback(q.name, _Rec(outs[q.name]))
    ih = rt.getInputHandler("StockStream")
    rt.start()
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=seed)
    offs = wl.call_offsets(n, call)
    ih.send_batch(ColumnBatch(ts, [sym, price, vol], [None, None, None], offs))
    rt.shutdown()
    return outs


def _same(a, b, rtol=1e-9):
    """Callback-for-callback equality; floating values (the window queries'
    segmented-scan averages) within 1e-9 relative, everything else exact."""
    if isinstance(a, float) and isinstance(b, float):
        return a == b or abs(a - b) <= rtol * max(abs(a), abs(b))
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(_same(x, y, rtol) for x, y in zip(a, b))
    return type(a) == type(b) and a == b


def test_m5_app_runs_on_oracle():
    """All 100 queries plan and run (checker side, small sample)."""
    outs = run_app(wl.M5_APP, OracleQueryEngine, 4000, 50, 0.05)
    assert len(outs) == 100
    assert sum(1 for v in outs.values() if v) >= 90


@pytest.mark.gpu
def test_m5_device_equals_oracle(hip_available):
    app = wl.M5_APP
    ora = run_app(app, OracleQueryEngine, 12000, 100, 0.02)
    dev = run_app(app, None, 12000, 100, 0.02)
    assert set(ora) == set(dev) and len(ora) == 100
    for name in ora:
        assert _same(dev[name], ora[name]), "query %s differs" % name
    assert sum(len(v) for v in ora.values()) > 0
