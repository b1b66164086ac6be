"""Batch windows on the device (window-x engine, engine_window.hip k_xb_*):
lengthBatch and timeBatch in full-batch mode, and the timeLength sliding
window (k_xw_time_lane with a length bound), against the oracle's restatement
of the processors, row for row (values, timestamps, types, callback chunks),
over several pushes: per-flush chunks of [expired previous batch] + RESET +
[current batch], the selector's batch picks (last per group, first-seen
order), RESET clearing every group state of the partition, timeBatch's
TIMER flushes (empty ones included) and start.time alignment, partitioned
lengthBatch, and the state through snapshot / restore.

Reference: C/query/processor/stream/window/LengthBatchWindowProcessor.java:153-243,
TimeBatchWindowProcessor.java:279-373, TimeLengthWindowProcessor.java:139-188,
C/util/Scheduler.java:71-220,
C/query/selector/QuerySelector.java:271-373,
C/query/selector/attribute/aggregator/AttributeAggregatorExecutor.java:144-150."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu

S = "@app:playback define stream S (symbol string, price float, volume int); "

APPS = [
    ("len-group", S + "@info(name = 'q') from S#window.lengthBatch(7) select symbol, sum(price) as s, "
     "count() as c group by symbol insert into O;"),
    ("len-all-avg", S + "@info(name = 'q') from S[volume > 20]#window.lengthBatch(5) select symbol, "
     "avg(price) as a, sum(volume) as v insert all events into O;"),
    ("len-plain-all", S + "@info(name = 'q') from S#window.lengthBatch(3) select symbol, price "
     "insert all events into O;"),
    ("len-having", S + "@info(name = 'q') from S#window.lengthBatch(9) select symbol, sum(price) as s "
     "group by symbol having s > 100.0 insert all events into O;"),
    ("len-expired-only", S + "@info(name = 'q') from S#window.lengthBatch(4) select symbol, count() as c "
     "group by symbol insert expired events into O;"),
    ("len-partitioned", S + "partition with (symbol of S) begin @info(name = 'q') from S#window.lengthBatch(3) "
     "select symbol, sum(price) as s, volume insert all events into O; end;"),
    ("len-part-group", S + "partition with (symbol of S) begin @info(name = 'q') from S#window.lengthBatch(4) "
     "select symbol, volume, count() as c group by volume insert into O; end;"),
    ("time-group", S + "@info(name = 'q') from S#window.timeBatch(1 sec) select symbol, sum(price) as s, "
     "avg(volume) as a group by symbol insert all events into O;"),
    ("time-plain", S + "@info(name = 'q') from S#window.timeBatch(700) select symbol, price "
     "insert all events into O;"),
    ("time-start", S + "@info(name = 'q') from S#window.timeBatch(2 sec, 0) select sum(price) as s, "
     "count() as c insert all events into O;"),
    ("time-current", S + "@info(name = 'q') from S[price > 40]#window.timeBatch(500) select symbol, "
     "sum(price) as m insert into O;"),
    # stream.current.event: events pass at once, the batch expires and RESETs later
    ("len-stream", S + "@info(name = 'q') from S#window.lengthBatch(5, true) select symbol, sum(price) as s "
     "group by symbol insert all events into O;"),
    ("len-stream-part", S + "partition with (symbol of S) begin @info(name = 'q') from S#window.lengthBatch(3, true) "
     "select symbol, price, count() as c insert all events into O; end;"),
    ("len-stream-plain", S + "@info(name = 'q') from S#window.lengthBatch(4, true) select symbol, price "
     "insert all events into O;"),
    ("len-zero", S + "@info(name = 'q') from S#window.lengthBatch(0) select symbol, sum(price) as s, count() as c "
     "group by symbol insert all events into O;"),
    ("time-stream", S + "@info(name = 'q') from S#window.timeBatch(1 sec, true) select symbol, sum(price) as s "
     "group by symbol insert all events into O;"),
    ("time-stream-start", S + "@info(name = 'q') from S#window.timeBatch(700, 100, true) select symbol, price "
     "insert all events into O;"),
    ("time-stream-cur", S + "@info(name = 'q') from S#window.timeBatch(500, true) select sum(price) as s, "
     "count() as c insert into O;"),
    # timeLength: a sliding window bounded by time and length (TIMER expiries too)
    ("timelen-group", S + "@info(name = 'q') from S#window.timeLength(2 sec, 5) select symbol, sum(price) as s "
     "group by symbol insert all events into O;"),
    ("timelen-time", S + "@info(name = 'q') from S#window.timeLength(3, 1000) select symbol, price, count() as c "
     "insert all events into O;"),
    ("timelen-part", S + "partition with (symbol of S) begin @info(name = 'q') from S#window.timeLength(1 sec, 3) "
     "select symbol, price, count() as c insert all events into O; end;"),
    ("timelen-plain", S + "@info(name = 'q') from S#window.timeLength(40, 60) select symbol, price "
     "insert expired events into O;"),
]


def gapped_batches(n, keys, seed, pushes=3, call=97):
    """StockStream rows 0.5 ms apart with two 4.5 s holes (TIMER flushes with
    nothing new: the previous batch expires alone)."""
    sym, price, vol, ts = wl.stock_stream(n, keys, 0.5, seed_offset=seed)
    price, vol = price.astype(np.float32), vol.astype(np.int32)   # the schema's float / int
    ts = ts.copy()
    ts[n // 3:] += 4500
    ts[2 * n // 3:] += 4500
    cut = np.linspace(0, n, pushes + 1).astype(int)
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call_size=call))
            for a, b in zip(cut[:-1], cut[1:])]


@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
def test_batch_window_equals_oracle(hip_available, name, app):
    qp, d = compile_single_query(app)
    wl.register_symbols(d, 12)
    batches = gapped_batches(12000, 12, seed=5)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_batch_window_single_event_calls(hip_available):
    """One event per InputHandler call: every lengthBatch flush and timeBatch
    TIMER lands in its own call."""
    for app in (APPS[1][1], APPS[7][1]):
        qp, d = compile_single_query(app)
        wl.register_symbols(d, 5)
        batches = gapped_batches(3000, 5, seed=8, pushes=2, call=1)
        ora = run_oracle(qp, batches)
        dev, _, _ = run_device(qp, batches)
        assert len(ora[2]) > 0
        assert_same_rows(dev, ora)


@pytest.mark.parametrize("idx", [1, 5, 7, 11, 12, 15])
def test_batch_window_snapshot_restore(hip_available, idx):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    qp, d = compile_single_query(APPS[idx][1])
    wl.register_symbols(d, 12)
    batches = gapped_batches(12000, 12, seed=6, pushes=4)
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


SE = "@app:playback define stream S (symbol string, price float, volume int, et long); "
EXT_APPS = [
    ("ext-group", SE + "@info(name = 'q') from S#window.externalTime(et, 30) select symbol, sum(price) as s "
     "group by symbol insert all events into O;"),
    ("ext-part", SE + "partition with (symbol of S) begin @info(name = 'q') from S#window.externalTime(et, 1 sec) "
     "select symbol, et, price insert all events into O; end;"),
    ("ext-plain", SE + "@info(name = 'q') from S[volume > 100]#window.externalTime(et, 7) select symbol, et "
     "insert expired events into O;"),
]


@pytest.mark.parametrize("name,app", EXT_APPS, ids=[a[0] for a in EXT_APPS])
def test_external_time_window_equals_oracle(hip_available, name, app):
    """externalTime: the window's clock is each event's own LONG attribute
    (here the arrival time plus a jitter of up to 6 ms, so it steps back now
    and then), no scheduler (ExternalTimeWindowProcessor.java:124-158)."""
    from siddhi_amd.runtime import ColumnBatch
    qp, d = compile_single_query(app)
    wl.register_symbols(d, 12)
    out = []
    for _, b in gapped_batches(12000, 12, seed=9):
        et = (b.ts + (b.cols[2] % 7)).astype(np.int64)
        out.append((0, ColumnBatch(b.ts, b.cols + [et], [None] * 4, b.call_offsets)))
    ora = run_oracle(qp, out)
    dev, _, _ = run_device(qp, out)
    assert len(ora[2]) > 0 and (ora[1] == 1).any()
    assert_same_rows(dev, ora)
