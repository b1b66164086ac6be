"""Block skipping in long pattern walks (k_block_sum + block_skippable,
siddhi_amd/csrc/engine_pattern.hip): a walk passes a whole 64-position block of
its key's sorted events when none of them can end it -- no f2 match (the
block's max / min of the compared e2 attribute against the partial's
threshold), no expiry, no time going back, no other key.  Rows must equal the
CPU oracle and the walk counters (partial_scans: (partial, event) pairs the
reference's pending-list scans visit) must equal the walks without skipping,
for >, >=, <, <= and a swapped comparison, both resume modes that walk long
(3: capped lane walks continued per wave; 2: one wave per partial), null e2
attributes, and a push whose events go back in time inside a key.

Reference: StreamPreStateProcessor.processAndReturn / expireEvents
(ST/StreamPreStateProcessor.java:326-403)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_oracle
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

SCHEMA = "@app:playback define stream S (symbol string, price double, volume long); "
F2 = {
    "gt": "price > e1.price * 1.05",
    "ge": "price >= e1.price * 1.05",
    "lt": "price < e1.price * 0.95",
    "le": "price <= e1.price * 0.95",
    "swapped": "e1.price * 1.05 < price",
}


def app(f2, f1="price > 60"):
    return (SCHEMA + "@info(name='q') from every e1=S[%s] -> e2=S[symbol == e1.symbol and %s] within 1 sec "
            "select e1.symbol as s, e1.price as p1, e2.price as p2 insert into O;" % (f1, f2))


def batches(n=30_000, keys=20, delta=0.05, parts=3, nulls=False, back=False, seed=4):
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=seed)
    pn = None
    if nulls:
        pn = (np.arange(n) % 11 == 3).astype(np.uint8)
    if back:
        ts = ts.copy()
        ts[n // 2:] -= 400        # the second half starts 400 ms before the first ended
    cuts = np.linspace(0, n, parts + 1).astype(int)
    out = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        offs = np.append(np.arange(0, b - a, 1024, dtype=np.int64), np.int64(b - a))
        out.append((0, ColumnBatch(ts[a:b], [sym[a:b], price[a:b], vol[a:b]],
                                   [None, None if pn is None else pn[a:b], None], offs)))
    return out


def run(qp, bs, monkeypatch, skip, mode):
    from parity import run_device
    monkeypatch.setenv("SHD_RESUME_MODE", mode)
    if skip:
        monkeypatch.setenv("SHD_BLOCK_SKIP", "1")
        monkeypatch.delenv("SHD_NO_BLOCK_SKIP", raising=False)
    else:
        monkeypatch.setenv("SHD_NO_BLOCK_SKIP", "1")
    dev, counters, kind = run_device(qp, bs)
    return dev, counters, kind


@pytest.mark.parametrize("mode", ["3", "2"])
@pytest.mark.parametrize("op", sorted(F2))
def test_block_skip_equals_oracle_and_counts(hip_available, monkeypatch, op, mode):
    qp, _ = compile_single_query(app(F2[op]))
    bs = batches(seed=len(op))
    ora = run_oracle(qp, bs)
    dev, c_skip, kind = run(qp, bs, monkeypatch, True, mode)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
    _, c_plain, _ = run(qp, bs, monkeypatch, False, mode)
    assert c_skip["partial_scans"] == c_plain["partial_scans"]
    assert c_skip["matches"] == c_plain["matches"] == len(ora[2])


def test_block_skip_null_e2_attributes(hip_available, monkeypatch):
    """Null prices never pass f2 and stay out of the block maxima."""
    qp, _ = compile_single_query(app(F2["gt"], f1="price > 50"))
    bs = batches(nulls=True, seed=9)
    ora = run_oracle(qp, bs)
    dev, c_skip, _ = run(qp, bs, monkeypatch, True, "3")
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)
    _, c_plain, _ = run(qp, bs, monkeypatch, False, "3")
    assert c_skip["partial_scans"] == c_plain["partial_scans"]


def test_block_skip_time_going_back(hip_available, monkeypatch):
    """A later push going back inside a key: the block's time flags keep the
    walks exact (the engine hands over to the NFA engine exactly as without
    skipping)."""
    qp, _ = compile_single_query(app(F2["gt"]))
    bs = batches(n=6_000, keys=30, delta=0.05, back=True, parts=2, seed=12)
    ora = run_oracle(qp, bs)
    dev, _, kind_skip = run(qp, bs, monkeypatch, True, "3")
    _, _, kind_plain = run(qp, bs, monkeypatch, False, "3")
    assert kind_skip == kind_plain
    assert_same_rows(dev, ora)


def test_m5_leader_shape_skips_by_default(hip_available, monkeypatch):
    """The M5 leader's density (~1000 same-symbol events per `within` span)
    turns skipping on without the test switch; rows equal the oracle."""
    from parity import run_device
    qp, _ = compile_single_query(app(F2["gt"]))
    bs = batches(n=20_000, keys=4, delta=0.1, parts=2, seed=21)
    ora = run_oracle(qp, bs)
    monkeypatch.delenv("SHD_BLOCK_SKIP", raising=False)
    monkeypatch.delenv("SHD_NO_BLOCK_SKIP", raising=False)
    dev, c, _ = run_device(qp, bs)
    assert_same_rows(dev, ora)
    monkeypatch.setenv("SHD_NO_BLOCK_SKIP", "1")
    _, c_plain, _ = run_device(qp, bs)
    assert c["partial_scans"] == c_plain["partial_scans"]
