"""The pattern engine's bucket walk (engine_bucket.hip k_bucket_walk, opt-in by
SHD_BUCKET_WALK=1; 2 also takes pushes that are not sparse): sparse
partitioned pushes sorted by 16 hashed key bits (two radix passes) and grouped
by key in LDS per bucket.  Against the CPU oracle row for row (values,
timestamps, callback chunks) over several pushes (carried partials), and
against the full-key sort path (the default) on the walk counters --
(partial, event) pairs visited, open partials carried -- which must not move.
Also: buckets beyond the LDS stage (skewed keys: the push re-runs on the
full-key sort), null partition keys (dropped events passed over), a
timestamp going back inside a key (hand-over to the generic NFA engine).

Reference: ST/StreamPreStateProcessor.java:118-129,326-403 (expiry, process),
C/partition/PartitionStreamReceiver.java:175-216 (null keys dropped)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu


def split(cols, parts, call=1024):
    sym, price, vol, ts = cols
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])
            if b > a]


@pytest.mark.parametrize("n,keys,delta,parts", [
    (400_000, 2_000_000, 0.01, 3),     # P3-like: 21-bit keys, almost every partial expires or stays open
    (300_000, 1 << 20, 0.0067, 4),     # E ~ 0.15: some walks meet their key inside `within` (matches)
    (250_000, 1_500_000, 0.02, 5),
])
def test_bucket_walk_equals_oracle_and_full_sort(hip_available, monkeypatch, n, keys, delta, parts):
    monkeypatch.setenv("SHD_BUCKET_WALK", "1")
    qp, _ = compile_single_query(wl.P3_APP)
    batches = split(wl.stock_stream(n, keys, delta, seed_offset=17), parts)
    ora = run_oracle(qp, batches)
    dev, c_bw, kind = run_device(qp, batches)
    assert kind == 1
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    monkeypatch.delenv("SHD_BUCKET_WALK")
    dev2, c_full, _ = run_device(qp, batches)
    assert_same_rows(dev2, ora)
    for k in ("events", "matches", "partials", "partial_scans", "carry"):
        assert c_bw[k] == c_full[k], k
    assert c_bw["group_bits"] == 16 and c_full["group_bits"] > 16


def test_bucket_overflow_reruns_on_the_full_sort(hip_available, monkeypatch):
    """Few keys: every bucket holds thousands of positions (beyond the LDS
    stage) -- forced onto the bucket walk, the push re-runs on the full-key
    sort and the rows stay the oracle's."""
    monkeypatch.setenv("SHD_BUCKET_WALK", "2")
    qp, _ = compile_single_query(wl.P3_APP)
    batches = split(wl.stock_stream(200_000, 40, 0.01, seed_offset=3), 2)
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_bucket_walk_small_keys_forced(hip_available, monkeypatch):
    """Forced onto the bucket walk with 15-bit keys (tiny buckets)."""
    monkeypatch.setenv("SHD_BUCKET_WALK", "2")
    qp, _ = compile_single_query(wl.P3_APP)
    batches = split(wl.stock_stream(200_000, 20_000, 0.01, seed_offset=4), 3)
    ora = run_oracle(qp, batches)
    dev, c, _ = run_device(qp, batches)
    assert c["group_bits"] == 16
    assert_same_rows(dev, ora)


def test_bucket_walk_null_keys(hip_available, monkeypatch):
    """Events with a null partition key are dropped (PartitionStreamReceiver);
    their rows sit in hashed buckets by row index and every walk passes over them."""
    monkeypatch.setenv("SHD_BUCKET_WALK", "1")
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(300_000, 2_000_000, 0.01, seed_offset=8)
    rng = np.random.default_rng(2)
    nul = (rng.random(len(ts)) < 0.03).astype(np.uint8)
    batches = []
    for a, b in ((0, 150_528), (150_528, len(ts))):
        offs = np.append(np.arange(0, b - a, 1024, dtype=np.int64), np.int64(b - a))
        batches.append((0, ColumnBatch(ts[a:b], [sym[a:b], price[a:b], vol[a:b]], [nul[a:b], None, None], offs)))
    ora = run_oracle(qp, batches)
    dev, c, _ = run_device(qp, batches)
    assert c["group_bits"] == 16
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_bucket_walk_time_regression_hands_over(hip_available, monkeypatch):
    """A push whose timestamps go back inside keys: the walk reports the
    violation and the query continues on the generic NFA engine."""
    monkeypatch.setenv("SHD_BUCKET_WALK", "1")
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(200_000, 1_000_000, 0.01, seed_offset=9)
    ts = ts.copy()
    ts[120_000:] -= 1500   # the second push starts 1.5 s before the first one ended
    batches = split((sym, price, vol, ts), 2)
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert kind == 4
    assert_same_rows(dev, ora)
