"""Pins, on the CPU, the reduction the device pattern engine relies on
(siddhi_amd/csrc/engine_pattern.hip header): for `every e1=A[f1] -> e2=B[f2]
within W` with per-key non-decreasing timestamps, partial P_i completes at the
first later B event j of its key with f2 before the first event with
ts - ts_i > W, and matches of one event come out in creation order.  Checked
against the object-graph oracle on seeded data."""
import numpy as np
import pytest

from parity import compile_single_query, run_oracle, stock_batch
from siddhi_amd import workloads as wl


def reduced(symbol, price, ts, within, partitioned, f1=lambda p: p > 70, factor=1.05):
    n = len(ts)
    by_key = {}
    order = np.arange(n)
    rows = []
    keys = symbol if partitioned else np.zeros(n, np.uint32)
    pos = {}
    for i in range(n):
        pos.setdefault(int(keys[i]), []).append(i)
    for k, idxs in pos.items():
        for a, i in enumerate(idxs):
            if not f1(price[i]):
                continue
            for j in idxs[a + 1:]:
                if ts[j] - ts[i] > within:
                    break
                if symbol[j] == symbol[i] and price[j] > price[i] * factor:
                    rows.append((j, i))
                    break
    rows.sort()
    return rows


@pytest.mark.parametrize("partitioned,n,keys,delta", [(False, 6000, 50, 1.0), (True, 20000, 2000, 0.05),
                                                      (True, 20000, 200, 1e-5)])
def test_forward_scan_reduction_equals_oracle(partitioned, n, keys, delta):
    app = wl.P3_APP if partitioned else wl.P1_APP
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=7)
    ora = run_oracle(qp, [(0, stock_batch(sym, price, vol, ts))])
    red = reduced(sym, price, ts, 1000, partitioned)
    assert len(red) == len(ora[2]) > 0
    # output columns: symbol, p1, p2 ; ts = ts_j
    exp_ts = np.array([ts[j] for j, i in red], np.int64)
    exp_p1 = np.array([price[i] for j, i in red])
    exp_p2 = np.array([price[j] for j, i in red])
    np.testing.assert_array_equal(ora[2], exp_ts)
    np.testing.assert_array_equal(ora[3][:, 1].view(np.float64), exp_p1)
    np.testing.assert_array_equal(ora[3][:, 2].view(np.float64), exp_p2)
