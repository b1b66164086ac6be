"""Time-sliced window aggregates on the device (the multi-GPU path of configs
W2-length / W2-time, siddhi_amd/exchange.py): the global stream is cut into
`world` contiguous slices; for each slice after the first, a fresh device query
is primed with the tail of the previous slice (the halo) -- its size found as
halo_take does, doubling until the query's carried window (counters.carry,
length) or the halo's time span (time) covers the window -- and its rows
dropped; then the slice is pushed.  The slices' rows concatenated must equal the
CPU oracle over the whole stream (doubles within 1e-9 relative, everything
else exact), for the call-window path (length, direct-mapped and hashed group
ids) and the segmented-scan path (time).  The rank-to-rank exchange itself is
covered with gloo in tests/test_window_slices.py."""
import numpy as np
import pytest
import torch

from parity import assert_rows_agg, compile_single_query, concat_rows, run_oracle, stock_batch
from siddhi_amd import exchange as ex
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu

CALL = 1024


def app(kind):
    win = "window.length(3000)" if kind == "length" else "window.time(200 millisec)"
    return ("@app:playback " + wl.STOCK_DEF + " @info(name='q') from StockStream[price>60]#%s "
            "select symbol, sum(price) as s, avg(volume) as a, count() as c group by symbol insert into O;" % win)


def push(dq, cols, ts):
    from siddhi_amd.hip_engine import SHD_MEM_HOST
    n = len(ts)
    offs = np.append(np.arange(0, n, CALL, dtype=np.int64), np.int64(n))
    cs = [np.ascontiguousarray(c) for c in cols]
    t = np.ascontiguousarray(ts, np.int64)
    dq.push_raw(0, n, t.ctypes.data, [c.ctypes.data for c in cs], [0, 0, 0], SHD_MEM_HOST,
                offs if len(offs) > 2 else None, True)


def prime(dq, prev, take, window, first_ts):
    """Fresh query, the halo (last `take` events of the previous slice) pushed
    and its rows dropped; True when it covers the window."""
    dq.reset()
    s, p, v, t = (c[-take:] for c in prev)
    push(dq, [s, p, v], t)
    dq.discard()
    return ex.halo_covers(window, dq.counters()["carry"], torch.from_numpy(t), first_ts)


@pytest.mark.parametrize("kind,keys", [("length", 40), ("length", 3000), ("time", 40)])
@pytest.mark.parametrize("world", [2, 3])
def test_sliced_device_rows_equal_whole_stream(hip_available, kind, keys, world):
    from siddhi_amd.hip_engine import DeviceQuery
    qp, _ = compile_single_query(app(kind))
    window = ex.window_of(qp)
    n = 12 * CALL + 300                           # every slice ends in a short call
    slices = [wl.stock_stream(n, keys, 0.05, seed_offset=8, start=r * n) for r in range(world)]
    whole = run_oracle(qp, [(0, stock_batch(*sl, CALL)) for sl in slices])
    assert len(whole[2]) > 0
    dq = DeviceQuery(qp.ir)
    parts, base, takes = [], 0, []
    try:
        for r, (s, p, v, t) in enumerate(slices):
            if r > 0:
                take = min(n, 2 * window[1] if kind == "length" else 4096)
                while not prime(dq, slices[r - 1], take, window, int(t[0])):
                    assert take < n, "window reaches past the previous slice"
                    take = min(n, 2 * take)
                takes.append(take)
            else:
                dq.reset()
            push(dq, [s, p, v], t)
            rows = dq.poll()
            if rows is not None:
                x = list(rows)
                x[0] = x[0] - x[0].min() + base     # chunk ids continue across slices
                base = int(x[0].max()) + 1
                parts.append(tuple(x))
    finally:
        dq.close()
    assert all(tk <= n for tk in takes)
    assert_rows_agg(concat_rows(parts), whole, qp, exact=False)


def test_short_halo_is_not_accepted(hip_available):
    """A halo holding fewer than L filter-passing events is refused (length)."""
    from siddhi_amd.hip_engine import DeviceQuery
    qp, _ = compile_single_query(app("length"))
    window = ex.window_of(qp)
    prev = wl.stock_stream(8 * CALL, 40, 0.05, seed_offset=8)
    dq = DeviceQuery(qp.ir)
    try:
        assert not prime(dq, prev, 3000, window, int(prev[3][-1]) + 1)   # ~80% of 3000 pass price > 60
        assert prime(dq, prev, 6000, window, int(prev[3][-1]) + 1)
        assert dq.counters()["carry"] == 3000
    finally:
        dq.close()
