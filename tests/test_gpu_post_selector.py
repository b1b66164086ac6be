"""Aggregating / `having` selectors over pattern and sequence output on the
device (state engine -> selector engine, the IR's POST section) against the
oracle's direct restatement of QuerySelector over StateEvents
(C/query/selector/QuerySelector.java:161-373, one StateEvent per chunk:
C/query/input/StateMultiProcessStreamReceiver.java:47-68), row for row and
bit-exact (the selector folds sequentially in emission order), over several
pushes; and the selector's aggregator state through snapshot / restore."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle
from test_post_selector import APPS, stream_batches
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
def test_device_equals_oracle(hip_available, name, app):
    qp, d = compile_single_query(app)
    wl.register_symbols(d, 50)
    batches = stream_batches(20000, 50, 0.5, seed=41)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_snapshot_restore_keeps_aggregates(hip_available):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, d = compile_single_query(APPS[1][1])
    wl.register_symbols(d, 50)
    batches = stream_batches(20000, 50, 0.5, seed=42, pushes=4)
    ora = run_oracle(qp, batches)

    def push(dq, b):
        cols = [np.ascontiguousarray(c) for c in b.cols]
        ts = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(0, b.n, ts.ctypes.data, [c.ctypes.data for c in cols], [0, 0, 0], SHD_MEM_HOST,
                    b.call_offsets, True)
        return dq.poll()

    dq = DeviceQuery(qp.ir)
    parts = [push(dq, batches[0][1]), push(dq, batches[1][1])]
    image = dq.snapshot()
    dq.close()
    dq2 = DeviceQuery(qp.ir)
    dq2.restore(image)
    parts += [push(dq2, batches[2][1]), push(dq2, batches[3][1])]
    dq2.close()
    dev = concat_rows([p for p in parts if p is not None])
    assert_same_rows(dev, ora)


MULTI_APPS = [
    ("seq-star", "@app:playback define stream S (symbol string, price float, volume int); "
     "@info(name = 'q') from every e1=S[(e1[last].price is null or e1[last].price <= price)]*, "
     "e2=S[price<e1[last].price] select e1.price as prices, e2.price as last, e1.volume as vols "
     "insert into O;"),
    ("pattern-count", "@app:playback define stream S (symbol string, price float, volume int); "
     "@info(name = 'q') from every e1=S[price>50]<2:4> -> e2=S[price<e1[0].price] "
     "select e1.symbol as syms, e1.price as prices, e2.price as p2 insert into O;"),
]


def _events(app, factory, sends):
    from siddhi_amd import runtime as rt
    mgr = rt.SiddhiManager(engine_factory=factory)
    r = mgr.createSiddhiAppRuntime(app)
    got = []

    class SC(rt.StreamCallback):
        def receive(self, events):
            got.append([(e.getTimestamp(), e.getData()) for e in events])
    r.addCallback("O", SC())
    r.start()
    h = r.getInputHandler("S")
    for ts, row in sends:
        h.send(ts, row)
    r.shutdown()
    return got


@pytest.mark.parametrize("name,app", MULTI_APPS, ids=[a[0] for a in MULTI_APPS])
def test_multi_value_selection_equals_oracle(hip_available, name, app):
    """`select e1.price` over a count state: a List per row
    (MultiValueVariableFunctionExecutor), device list arena == oracle."""
    from oracle_engine import OracleQueryEngine
    from siddhi_amd.hip_engine import HipQueryEngine
    rng = np.random.default_rng(7)
    sends = [(1000 + i, ["S%d" % rng.integers(0, 4), float(np.float32(rng.uniform(20, 80))),
                         int(rng.integers(0, 100))]) for i in range(3000)]
    ora = _events(app, OracleQueryEngine, sends)
    dev = _events(app, HipQueryEngine, sends)
    assert sum(len(c) for c in ora) > 10
    assert any(len(d[0]) > 1 for c in ora for _, d in c)   # lists with several elements
    assert dev == ora
