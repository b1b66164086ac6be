"""The bucketed time-local walk of the pattern engine (engine_pattern.hip,
k_bkt_walk: one hashed pass into 256 buckets, chunks of a bucket staged in
LDS with their `within` lookahead, partials resolved against their key's
later events there) against the CPU oracle and against the device's sort
path, on the P1 query shape: the walk retires partials at the push horizon,
which only global expiry (unpartitioned plans) makes exact -- partitioned
plans (P3) never take it and must still equal the oracle when it is asked
for.  Covers carried partials across pushes,
null partition keys (dropped events), lookahead overflow (dense keys: the
walk continues in HBM), retired partials, and pushes that are not
time-ordered (redone on the sort path)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu


def _split(cols, parts, call=1024):
    sym, price, vol, ts = cols
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)) for a, b in zip(cuts[:-1], cuts[1:])
            if b > a]


CASES = [
    # name, app, events, keys, delta ms
    ("P3-sparse", wl.P3_APP, 240_000, 50_000, 0.01),
    ("P3-mid", wl.P3_APP, 200_000, 3_000, 0.02),
    ("P3-dense-overflow", wl.P3_APP, 200_000, 2_000, 1e-4),   # bucket span > lookahead: HBM walk
    ("P1-implicit", wl.P1_APP, 150_000, 1_000, 0.05),
]


@pytest.mark.parametrize("parts", [1, 4])
@pytest.mark.parametrize("name,app,n,keys,delta", CASES, ids=[c[0] for c in CASES])
def test_bucket_walk_equals_oracle(hip_available, monkeypatch, name, app, n, keys, delta, parts):
    monkeypatch.setenv("SHD_BUCKET", "1")
    qp, _ = compile_single_query(app)
    batches = _split(wl.stock_stream(n, keys, delta, seed_offset=hash(name) % 997), parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
    if name.startswith("P3"):
        assert counters["group_bits"] != 8   # partitioned: never the (retiring) bucketed walk
    else:
        assert counters["group_bits"] == 8   # the bucketed walk ran
    monkeypatch.setenv("SHD_NO_BUCKET", "1")
    dev2, c2, _ = run_device(qp, batches)
    assert_same_rows(dev2, ora)


def test_bucket_walk_null_keys_and_strings(hip_available, monkeypatch):
    """Partition key with nulls (PartitionStreamReceiver drops those events)."""
    monkeypatch.setenv("SHD_BUCKET", "1")
    app = ("@app:playback define stream S (k string, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>40] -> e2=S[p>e1.p] within 3 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(12)
    n = 150_000
    k = rng.integers(0, 20_000, n).astype(np.uint32)
    kn = (rng.random(n) < 0.03).astype(np.uint8)
    p = rng.uniform(0, 100, n)
    ts = 10_000 + np.arange(n, dtype=np.int64) // 20
    batches = [(0, ColumnBatch(ts[a:b], [k[a:b], p[a:b]], [kn[a:b], None], np.arange(a, b + 1, 1000) - a))
               for a, b in ((0, 70_000), (70_000, n))]
    ora = run_oracle(qp, batches)
    dev, counters, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["group_bits"] != 8


def test_bucket_walk_redoes_unordered_push(hip_available, monkeypatch):
    """A push whose events are not globally time-ordered (per-key order kept)
    is redone on the sort path; the result is still the oracle's."""
    monkeypatch.setenv("SHD_BUCKET", "1")
    app = ("@app:playback define stream S (k int, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>50] -> e2=S[p>e1.p] within 30 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(3)
    n = 100_000
    k = rng.integers(0, 3000, n).astype(np.int32)
    p = rng.uniform(0, 100, n)
    ts = 1_000_000 + np.arange(n, dtype=np.int64) // 8 + (k.astype(np.int64) % 5) * 40
    batches = [(0, ColumnBatch(ts, [k, p], [None, None], np.arange(0, n + 1, 1000)))]
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["group_bits"] != 8   # not the bucketed walk
