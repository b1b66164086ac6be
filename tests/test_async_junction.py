"""`@Async(buffer.size, workers, batch.size.max)` stream definitions (SURVEY.md
§8f rank 4; C/stream/StreamJunction.java:250-306, StreamHandler).

The reference publishes each event into a disruptor ring and worker threads
hand the receivers batches of at most batch.size.max events; which batches
form depends on thread timing, so the reference's own tests
(T/managment/AsyncTestCase.java asyncTest3-5) assert only the event counts and
the batch bound.  This runtime accepts the annotation and delivers each
publish as its own batch, in publish order -- the schedule the disruptor
produces when its consumers keep up -- so those assertions hold; the
per-worker thread counts they also log (asyncTest4: two worker threads) have
no counterpart in a synchronous runtime and are not restated.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle_engine import OracleQueryEngine  # noqa: E402
from siddhi_amd.runtime import SiddhiManager, StreamCallback  # noqa: E402

APP3 = ("@async(buffer.size='2')"
        "define stream cseEventStream (symbol string, price float, volume int);"
        "define stream cseEventStream2 (symbol string, price float, volume int);"
        "@info(name = 'query1') from cseEventStream[70 > price] select * insert into innerStream ;"
        "@info(name = 'query2') from innerStream[volume > 90] select * insert into outputStream ;")
APP4 = ("@async(buffer.size='16', workers='2', batch.size.max='2')"
        "define stream cseEventStream (symbol string, price float, volume int);"
        "@info(name = 'query1') from cseEventStream[70 < price] select * insert into innerStream ;"
        "@info(name = 'query2') from innerStream[volume > 90] select * insert into outputStream ;")
APP5 = ("@async(buffer.size='512', workers='10', batch.size.max='20')"
        "define stream cseEventStream (symbol string, price float, volume int);"
        "@info(name = 'query1') from cseEventStream[70 < price] select * insert into outputStream ;")


def _run(app, sends, device):
    m = SiddhiManager() if device else SiddhiManager(engine_factory=OracleQueryEngine)
    rt = m.createSiddhiAppRuntime(app)
    batches = []

    class CB(StreamCallback):
        def receive(self, events):
            batches.append([list(e.data) for e in events])

    rt.addCallback("outputStream", CB())
    rt.start()
    ih = rt.getInputHandler("cseEventStream")
    for d in sends:
        ih.send(d)
    rt.shutdown()
    return batches


def _cases(device):
    # asyncTest3: 5 events pass both filters
    b = _run(APP3, [["WSO2", 55.6, 100], ["IBM", 9.6, 100], ["FB", 7.6, 100], ["GOOG", 5.6, 100],
                    ["WSO2", 15.6, 100]], device)
    assert sum(len(x) for x in b) == 5
    # asyncTest4: 20 events, batches of at most batch.size.max = 2
    b = _run(APP4, [["WSO2", 115.6, 100 + i] for i in range(20)], device)
    assert sum(len(x) for x in b) == 20 and all(len(x) <= 2 for x in b)
    assert [x[2] for y in b for x in y] == [100 + i for i in range(20)]   # publish order
    # asyncTest5: 1200 events, batches of at most 20
    b = _run(APP5, [["WSO2", 115.6, 100 + i] for i in range(1200)], device)
    assert sum(len(x) for x in b) == 1200 and all(len(x) <= 20 for x in b)


def test_async_streams_oracle():
    _cases(False)


@pytest.mark.gpu
def test_async_streams_device(hip_available):
    _cases(True)
