"""Device (libsiddhi_hip on MI355X) vs CPU oracle on seeded StockStream
workloads (configs P1, P3, W2 at oracle-sized scale), including micro-batch
splits that exercise the carried partial-match / window state.
Integer/index/string/timestamp outputs must be bit-exact; double aggregates
are bit-exact in the `exact_aggregates` mode (sequential per-group fold) and
within 1e-9 relative in the default segmented-scan mode."""
import numpy as np
import pytest

from parity import assert_rows_agg, assert_same_rows, compile_single_query, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu


def split(sym, price, vol, ts, parts, call=1024):
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    out = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b > a:
            out.append((0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)))
    return out


CASES = [
    ("P1", wl.P1_APP, 30000, 1000, 1.0),
    ("P1-denser", wl.P1_APP, 30000, 50, 0.2),
    ("P3", wl.P3_APP, 200000, 20000, 0.01),
    ("P3-dense", wl.P3_APP, 200000, 20000, 1e-5),
    ("W2-length", wl.W2_LENGTH_APP, 100000, 1000, 0.1),
    ("W2-time", wl.W2_TIME_APP, 100000, 1000, 0.5),
    ("W2-time-short", wl.W2_TIME_APP.replace("10 sec", "40 milliseconds"), 50000, 100, 0.5),
]


@pytest.mark.parametrize("name,app,n,keys,delta", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("parts", [1, 3])
@pytest.mark.parametrize("mode", ["scan", "exact"])
def test_device_equals_oracle(hip_available, name, app, n, keys, delta, parts, mode):
    if mode == "exact" and not name.startswith("W2"):
        pytest.skip("exact_aggregates only concerns window aggregates")
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=hash(name) % 1000)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches, exact=mode == "exact")
    assert len(ora[2]) > 0
    assert_rows_agg(dev, ora, qp, mode == "exact")
    assert counters["events"] == n


@pytest.mark.parametrize("mode", ["scan", "exact"])
def test_single_event_calls_match_oracle(hip_available, mode):
    # B = 1 variant: every InputHandler call carries one event
    qp, _ = compile_single_query(wl.W2_LENGTH_APP.replace("length(1000)", "length(7)"))
    sym, price, vol, ts = wl.stock_stream(3000, 13, 1.0, seed_offset=3)
    batches = [(0, stock_batch(sym, price, vol, ts, call_size=1))]
    assert_rows_agg(run_device(qp, batches, exact=mode == "exact")[0], run_oracle(qp, batches), qp,
                    mode == "exact")


def test_two_stream_pattern_matches_oracle(hip_available):
    app = ("define stream A (k int, p double); define stream B (k int, p double); "
           "partition with (k of A, k of B) begin "
           "@info(name='q') from every e1=A[p>20] -> e2=B[p>e1.p] within 50 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(5)
    batches = []
    t = 1000
    for r in range(40):
        si = int(rng.integers(0, 2))
        m = int(rng.integers(1, 300))
        k = rng.integers(0, 30, m).astype(np.int32)
        p = rng.uniform(0, 100, m)
        ts = t + np.sort(rng.integers(0, 20, m)).astype(np.int64)
        t = int(ts[-1])
        batches.append((si, ColumnBatch(ts, [k, p], [None, None], np.array([0, m], np.int64))))
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_partitioned_open_partials_survive_time_going_back(hip_available):
    """A partitioned partial is expired only by an event of its own key
    (per-key pending lists, StreamPreStateProcessor.expireEvents :326-361), so
    the device carries every open partial across pushes -- nothing is retired
    at a global time horizon -- and a later push whose events go back before
    earlier pushes' times still meets them exactly as the reference does (the
    pushes are large enough that unpartitioned plans would retire partials)."""
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(300_000, 100_000, 0.05, seed_offset=41)
    batches = split(sym, price, vol, ts, 3)
    # a fourth push replays the first push's events: every timestamp precedes
    # the third push's, and its keys meet partials carried from all three
    batches.append(batches[0])
    ora = run_oracle(qp, batches)
    dev, counters, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["events"] == sum(b.n for _, b in batches)


def test_unpartitioned_retirement_then_time_going_back(hip_available):
    """Unpartitioned plans expire globally: partials the last event of a push
    expired are gone in the reference too and may be retired; a later push that
    goes back before that time continues on the generic NFA engine (the open
    partials handed over) and equals the oracle."""
    qp, _ = compile_single_query(wl.P1_APP.replace("within 1 sec", "within 20 milliseconds"))
    sym, price, vol, ts = wl.stock_stream(210_000, 200, 0.01, seed_offset=43)
    batches = split(sym, price, vol, ts, 3)
    batches.append((0, stock_batch(sym[:5000], price[:5000], vol[:5000], ts[:5000] + 300)))
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("within", ["within 40 days", ""])
def test_timestamps_beyond_32bit_offsets(hip_available, within):
    """Timestamps travel with the key sort as 32-bit offsets from the batch's
    first event; a batch spanning more than 2^31 ms (with or without `within`)
    takes the 64-bit path and must give the same matches."""
    app = ("define stream S (k int, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>50] -> e2=S[p>e1.p] " + within +
           " select e1.k as k, e1.p as p1, e2.p as p2, e2.p - e1.p as d insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(17)
    n = 20000
    k = rng.integers(0, 500, n).astype(np.int32)
    p = rng.uniform(0, 100, n)
    ts = 1_600_000_000_000 + np.cumsum(rng.integers(0, 400_000, n)).astype(np.int64)   # ~46 days
    assert ts[-1] - ts[0] > 2 ** 31
    batches = [(0, ColumnBatch(ts[a:b], [k[a:b], p[a:b]], [None, None], np.arange(a, b + 1, 1000) - a))
               for a, b in ((0, 7000), (7000, n))]
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("keys", [40, 100_000])
@pytest.mark.parametrize("parts", [1, 3])
def test_partitioned_key_sort(hip_available, keys, parts):
    """Partitioned P3 on the full key sort + forward scan: 100k keys (17 key
    bits) and 40 keys (every key holds thousands of rows), equal to the
    oracle."""
    qp, _ = compile_single_query(wl.P3_APP)
    n = 300_000
    sym, price, vol, ts = wl.stock_stream(n, keys, 0.01, seed_offset=77)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["group_bits"] == (17 if keys == 100_000 else 6)


def test_hashed_grouping_needs_time_order(hip_available, monkeypatch):
    """Pushed rows that are not globally time-ordered (per-key order intact)
    keep the exact key sort even when hashed buckets are requested."""
    monkeypatch.setenv("SHD_HASH_BITS", "8")
    app = ("define stream S (k int, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>50] -> e2=S[p>e1.p] within 30 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(23)
    n = 100_000
    k = rng.integers(0, 3000, n).astype(np.int32)
    p = rng.uniform(0, 100, n)
    # per key non-decreasing, globally not: key-dependent clock offsets
    ts = 1_000_000 + np.arange(n, dtype=np.int64) // 4 + (k.astype(np.int64) % 7) * 50
    batches = [(0, ColumnBatch(ts, [k, p], [None, None], np.arange(0, n + 1, 1000)))]
    ora = run_oracle(qp, batches)
    dev, counters, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    # exact grouping: the full key sort (12 bits) or the grouped LDS walk (16
    # hashed bits, every row of a key in one group) -- never partial buckets
    assert counters["group_bits"] in (12, 16)


@pytest.mark.parametrize("implicit", [True, False])
@pytest.mark.parametrize("parts", [1, 3])
def test_unpartitioned_pattern_grouped_by_equality(hip_available, monkeypatch, implicit, parts):
    """Config P1 (unpartitioned, f2 holds `symbol == e1.symbol`): with
    time-ordered events the engine groups by symbol like a partitioned query
    (SHD_NO_IMPLICIT_KEY turns that off); results identical to the oracle."""
    if not implicit:
        monkeypatch.setenv("SHD_NO_IMPLICIT_KEY", "1")
    qp, _ = compile_single_query(wl.P1_APP)
    sym, price, vol, ts = wl.stock_stream(100_000, 1000, 0.5, seed_offset=91)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert (counters["group_bits"] > 0) == implicit


@pytest.mark.parametrize("reverse", [False, True])
def test_implicit_grouping_edge_cases(hip_available, reverse):
    """Null symbols and two streams keyed by their own attribute; with
    `reverse`, one push whose events go back in time inside a key (the query
    hands over to the generic NFA engine and still equals the oracle)."""
    app = ("@app:playback define stream A (k string, p double); define stream B (k string, p double); "
           "@info(name='q') from every e1=A[p>20] -> e2=B[k==e1.k and p>e1.p] within 50 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O;")
    qp, d = compile_single_query(app)
    rng = np.random.default_rng(8)
    batches = []
    t = 1000
    for r in range(30):
        si = r % 2
        m = int(rng.integers(1000, 6000))
        k = rng.integers(0, 40, m).astype(np.uint32)
        kn = (rng.random(m) < 0.05).astype(np.uint8)   # null keys
        p = rng.uniform(0, 100, m)
        ts = t + np.sort(rng.integers(0, 30, m)).astype(np.int64)
        if reverse and r == 17:
            ts = ts[::-1].copy()   # time goes back inside this push
        t = int(ts.max())
        batches.append((si, ColumnBatch(ts, [k, p], [kn, None], np.array([0, m], np.int64))))
    ora = run_oracle(qp, batches)
    assert len(ora[2]) > 0
    dev, _, kind = run_device(qp, batches)
    assert_same_rows(dev, ora)
    assert kind == (4 if reverse else 1)


TYPED_WINDOW_APPS = [
    ("length-sum-avg-count", "define stream S (k int, i int, l long, f float, d double); @info(name='q') "
     "from S[d > -1.0]#window.length(300) select k, sum(i) as si, sum(l) as sl, avg(f) as af, count() as c "
     "group by k insert into O;"),
    ("time-sum-avg", "define stream S (k int, i int, l long, f float, d double); @info(name='q') "
     "from S#window.time(40 milliseconds) select k, sum(d) as sd, avg(d) as ad, sum(f) as sf "
     "group by k insert into O;"),
    ("length-w2-shape", "define stream S (k int, i int, l long, f float, d double); @info(name='q') "
     "from S[d > 20.0]#window.length(700) select k, avg(d) as a, sum(d) as s, count() as c, avg(i) as ai "
     "group by k insert into O;"),
]


@pytest.mark.parametrize("fold", ["wave", "wave-generic", "lane", "scan"])
@pytest.mark.parametrize("name,app", TYPED_WINDOW_APPS, ids=[a[0] for a in TYPED_WINDOW_APPS])
def test_group_fold_long_segments(hip_available, monkeypatch, fold, name, app):
    """Few groups, long operation segments per push: the one-wave-per-group
    fold (coalesced operand loads, wave-uniform sequential state) and the
    one-lane-per-group fold must both give the oracle's rows bit for bit,
    typed aggregates and null arguments included; the segmented-scan mode
    (default; integer sums stay on the fold) within 1e-9 relative."""
    if fold == "lane":
        monkeypatch.setenv("SHD_FOLD_LANE", "1")
    if fold == "wave-generic":
        monkeypatch.setenv("SHD_FOLD_GENERIC", "1")
    qp, _ = compile_single_query("@app:playback " + app)
    rng = np.random.default_rng(31)
    batches = []
    t = 10_000
    for r in range(4):
        m = 30_000
        k = rng.integers(0, 6, m).astype(np.int32)
        i = rng.integers(-1000, 1000, m).astype(np.int32)
        lv = rng.integers(-10 ** 12, 10 ** 12, m).astype(np.int64)
        f = rng.uniform(-50, 50, m).astype(np.float32)
        d = rng.uniform(0, 100, m)
        nulls = [None, (rng.random(m) < 0.03).astype(np.uint8), None, (rng.random(m) < 0.03).astype(np.uint8),
                 (rng.random(m) < 0.03).astype(np.uint8)]
        ts = t + np.sort(rng.integers(0, 3000, m)).astype(np.int64)
        t = int(ts[-1])
        batches.append((0, ColumnBatch(ts, [k, i, lv, f, d], nulls, np.arange(0, m + 1, 500, dtype=np.int64))))
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches, exact=fold != "scan")
    assert len(ora[2]) > 0
    assert_rows_agg(dev, ora, qp, fold != "scan")


@pytest.mark.parametrize("parts", [1, 3])
def test_partition_keys_far_from_zero(hip_available, parts):
    """Keys of a push span [kmin, kmax] far from 0 (one rank's key slice):
    the full key sort covers only the bits of kmax - kmin; rows of null-key
    events (dropped by PartitionStreamReceiver) sit anywhere in the sorted
    order and are passed over by the walks."""
    app = ("define stream S (k int, p double); partition with (k of S) begin "
           "@info(name='q') from every e1=S[p>40] -> e2=S[p>e1.p*1.02] within 30 milliseconds "
           "select e1.k as k, e1.p as p1, e2.p as p2 insert into O; end;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(12)
    n = 120_000
    k = (70_000_000 + rng.integers(0, 20_000, n)).astype(np.int32)
    kn = (rng.random(n) < 0.05).astype(np.uint8)
    k[kn.astype(bool)] = 0
    p = rng.uniform(0, 100, n)
    ts = 5_000 + np.arange(n, dtype=np.int64) // 20
    cuts = [int(n * j / parts) for j in range(parts + 1)]
    batches = [(0, ColumnBatch(ts[a:b], [k[a:b], p[a:b]], [kn[a:b], None], np.arange(a, b + 1, 1000) - a))
               for a, b in zip(cuts[:-1], cuts[1:])]
    ora = run_oracle(qp, batches)
    dev, counters, _ = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert counters["group_bits"] == 15


@pytest.mark.parametrize("back", [False, True])
def test_sparse_keys_carry_and_go_back(hip_available, back):
    """Partitioned P3 with sparse keys (the bench's shape): every open partial
    is carried until an event of its key expires or completes it (per-key
    expiry, StreamPreStateProcessor.expireEvents :326-361).  With `back`, a
    last push goes back in time: the open partials are handed to the NFA
    engine.  Equal to the oracle either way."""
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(240_000, 60_000, 0.05, seed_offset=53)
    batches = split(sym, price, vol, ts, 6)
    if back:
        batches.append(batches[1])
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    assert kind == (4 if back else 1)
    if not back:
        assert counters["carry"] > 0


@pytest.mark.parametrize("shape", ["sparse", "dense"])
@pytest.mark.parametrize("parts", [1, 4])
def test_p3_shapes(hip_available, shape, parts):
    """Partitioned P3 over sparse (the bench's 10 events / key / `within`
    fraction) and dense keys, in one push or four: equal to the oracle."""
    qp, _ = compile_single_query(wl.P3_APP)
    n, keys, delta = (240_000, 60_000, 0.05) if shape == "sparse" else (200_000, 2_000, 0.002)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=71)
    batches = split(sym, price, vol, ts, parts)
    ora = run_oracle(qp, batches)
    dev, counters, kind = run_device(qp, batches)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
