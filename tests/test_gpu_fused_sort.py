"""The pattern engine's fused row preparation + first key-sort pass
(keyed_sort.hip; partitioned plans on a 32-bit plain key, the P3 default from
1 M extended rows per push, forced here with SHD_FUSED_SORT=1 at test sizes).
Against the CPU oracle row for row (values, timestamps, callback chunks) over
several pushes (carried partials), and against the unfused path
(SHD_FUSED_SORT=0: k_prepare + a full radix sort) on the walk counters --
candidates created, (partial, event) pairs visited, open partials carried --
which must not move.  Shapes: P3-like sparse keys, keys far from 0 (the sort
runs on key - kmin), key ranges of one digit and of a single key (no sort),
null partition keys (dropped rows keyed by their row index), f1 on int / float
/ long attributes and without a filter, and a time regression (hand-over to
the generic NFA engine).

Reference: ST/StreamPreStateProcessor.java:118-129,326-403 (expiry, process),
C/partition/PartitionStreamReceiver.java:175-216 (null keys dropped)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle, stock_batch
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

COUNTERS = ("events", "matches", "partials", "partial_scans", "carry")


def split(cols, parts, call=1024, nulls=None):
    sym, price, vol, ts = cols
    n = len(ts)
    cuts = sorted(set([0, n] + [int(n * k / parts) // call * call for k in range(1, parts)]))
    out = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b <= a:
            continue
        if nulls is None:
            out.append((0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], call)))
        else:
            offs = np.append(np.arange(0, b - a, call, dtype=np.int64), np.int64(b - a))
            out.append((0, ColumnBatch(ts[a:b], [sym[a:b], price[a:b], vol[a:b]],
                                       [None if x is None else x[a:b] for x in nulls], offs)))
    return out


def check(qp, batches, monkeypatch, min_rows=1):
    ora = run_oracle(qp, batches)
    assert len(ora[2]) >= min_rows
    monkeypatch.setenv("SHD_FUSED_SORT", "1")
    dev, c_f, kind = run_device(qp, batches)
    assert_same_rows(dev, ora)
    monkeypatch.setenv("SHD_FUSED_SORT", "0")
    dev2, c_u, kind2 = run_device(qp, batches)
    assert_same_rows(dev2, ora)
    if kind == 1 and kind2 == 1:
        for k in COUNTERS:
            assert c_f[k] == c_u[k], k
        assert c_f["group_bits"] == c_u["group_bits"]
    return c_f, kind


@pytest.mark.parametrize("n,keys,delta,parts,base", [
    (400_000, 2_000_000, 0.01, 3, 0),          # P3-like: almost every partial expires or stays open
    (300_000, 1 << 20, 0.0067, 4, 0),          # some walks meet their key inside `within` (matches)
    (250_000, 1_500_000, 0.02, 5, 70_000_000),  # keys far from 0: digits of key - kmin
    (200_000, 40, 0.01, 2, 0),                 # one digit: the fused pass is the whole sort
    (120_000, 300, 0.01, 3, 255),              # kmin's low byte != 0: the first digit is rotated
])
def test_fused_sort_equals_oracle_and_unfused(hip_available, monkeypatch, n, keys, delta, parts, base):
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=17)
    sym = (sym + np.uint32(base)).astype(np.uint32)
    c, kind = check(qp, split((sym, price, vol, ts), parts), monkeypatch)
    assert kind == 1


def test_fused_sort_single_key_and_null_keys(hip_available, monkeypatch):
    """All events on one key (a zero-width sort: no pass reorders anything)
    plus null keys, whose rows carry their row index as key."""
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(60_000, 1, 0.5, seed_offset=5)
    rng = np.random.default_rng(3)
    nul = (rng.random(len(ts)) < 0.05).astype(np.uint8)
    check(qp, split((sym, price, vol, ts), 2, nulls=[nul, None, None]), monkeypatch)


def test_fused_sort_null_keys_and_null_operands(hip_available, monkeypatch):
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(300_000, 1 << 18, 0.002, seed_offset=8)
    rng = np.random.default_rng(2)
    knul = (rng.random(len(ts)) < 0.03).astype(np.uint8)
    pnul = (rng.random(len(ts)) < 0.02).astype(np.uint8)
    check(qp, split((sym, price, vol, ts), 3, nulls=[knul, pnul, None]), monkeypatch)


@pytest.mark.parametrize("schema,f1", [
    ("symbol string, price float, volume int", "volume > 400"),
    ("symbol string, price float, volume int", "price > 70"),
    ("symbol string, price double, volume long", "volume >= 500"),
    ("symbol string, price double, volume long", None),
    ("symbol int, price double, volume long", "price > 70"),
])
def test_fused_sort_f1_types(hip_available, monkeypatch, schema, f1):
    app = ("@app:playback define stream S (%s); partition with (symbol of S) begin "
           "@info(name='q') from every e1=S%s -> e2=S[symbol == e1.symbol and price > e1.price * 1.05] "
           "within 1 sec select e1.symbol as s, e1.price as p1, e2.price as p2 insert into O; end;"
           % (schema, "" if f1 is None else "[" + f1 + "]"))
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(200_000, 1 << 16, 0.005, seed_offset=21)
    if "price float" in schema:
        price = price.astype(np.float32)
    if "volume int" in schema:
        vol = (vol % 1000).astype(np.int32)
    if "symbol int" in schema:
        sym = sym.astype(np.int32)
    check(qp, split((sym, price, vol, ts), 2), monkeypatch)


def test_fused_sort_time_regression_hands_over(hip_available, monkeypatch):
    """A push whose timestamps go back inside keys: the walk reports the
    violation and the query continues on the generic NFA engine."""
    qp, _ = compile_single_query(wl.P3_APP)
    sym, price, vol, ts = wl.stock_stream(200_000, 1_000_000, 0.01, seed_offset=9)
    ts = ts.copy()
    ts[120_000:] -= 1500   # the second push starts 1.5 s before the first one ended
    batches = split((sym, price, vol, ts), 2)
    ora = run_oracle(qp, batches)
    monkeypatch.setenv("SHD_FUSED_SORT", "1")
    dev, _, kind = run_device(qp, batches)
    assert kind == 4
    assert_same_rows(dev, ora)


@pytest.mark.parametrize("f1", ["price > 70", "70 <= price", "price != 70.5", "price < 60 ", "price == 50"])
def test_fused_sort_f1_resolved_and_generic(hip_available, monkeypatch, f1):
    """f1 on a double column against a constant runs pre-resolved in the fused
    pass (operator outside the row loop, swapped operands flipped); the same
    pushes through eval_fpred per row (SHD_KS_GENERIC_F1) give the same rows."""
    app = wl.P3_APP.replace("StockStream[price>70]", "StockStream[%s]" % f1)
    assert app != wl.P3_APP or f1 == "price > 70"
    qp, _ = compile_single_query(app)
    sym, price, vol, ts = wl.stock_stream(150_000, 1 << 15, 0.005, seed_offset=23)
    price = np.round(price * 2) / 2   # some prices equal the constants
    rng = np.random.default_rng(5)
    pnul = (rng.random(len(ts)) < 0.02).astype(np.uint8)
    batches = split((sym, price, vol, ts), 2, nulls=[None, pnul, None])
    check(qp, batches, monkeypatch, min_rows=0)
    monkeypatch.setenv("SHD_KS_GENERIC_F1", "1")
    check(qp, batches, monkeypatch, min_rows=0)


@pytest.mark.parametrize("app,keys", [("P3", 1_500_000), ("and", 1_500_000), ("or", 4_000_000)])
def test_resume_list_equals_tile_pass(hip_available, monkeypatch, app, keys):
    """Sparse keys: the deferred walks run from a compacted list, one lane each
    (k_resume_list), instead of the per-tile outcome-byte pass (MODE 0,
    SHD_NO_RESUME_LIST): same rows as the oracle, same walk counters."""
    text = wl.P3_APP if app == "P3" else wl.S4_PART_APPS[app]
    qp, _ = compile_single_query(text)
    # E = events of a partial's key inside `within` < 0.25: the sparse layout
    sym, price, vol, ts = wl.stock_stream(400_000, keys, 0.01, seed_offset=29)
    batches = split((sym, price, vol, ts), 3)
    ora = run_oracle(qp, batches)
    assert len(ora[2]) > 0
    monkeypatch.delenv("SHD_NO_RESUME_LIST", raising=False)
    dev, c_list, kind = run_device(qp, batches)
    assert kind == 1
    assert_same_rows(dev, ora)
    monkeypatch.setenv("SHD_NO_RESUME_LIST", "1")
    dev2, c_tile, _ = run_device(qp, batches)
    assert_same_rows(dev2, ora)
    for k in COUNTERS:
        assert c_list[k] == c_tile[k], k
