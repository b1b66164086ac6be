"""Lockstep pattern walks and the split f2 (k_lockstep_walk, siddhi_amd/csrc/engine_pattern.hip,
the default for dense keys; SHD_LOCKSTEP=1 / 0 forces it on / off): f2 evaluated inside the one-lane-per-position walk,
every candidate of a wave advancing one sorted position per round, walks past
64 positions continued by the wave-cooperative pass (PS_CONT).  Rows must
equal the CPU oracle and the walk counters (partial_scans, matches) the
hot-walk + deferred-walk path's, for sparse keys, dense keys with
walks beyond the 64-position cap, null e2 attributes and a push going back
in time inside a key.

Reference: StreamPreStateProcessor.processAndReturn / expireEvents
(ST/StreamPreStateProcessor.java:326-403)."""
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle
from test_gpu_block_skip import F2, app, batches

pytestmark = pytest.mark.gpu

CASES = {
    "sparse": dict(n=30_000, keys=20_000, delta=0.5),
    "dense": dict(n=30_000, keys=2_000, delta=0.05),
    "long": dict(n=30_000, keys=400, delta=0.05),     # walks beyond the 64-position cap
}


def run(qp, bs, monkeypatch, lockstep):
    monkeypatch.setenv("SHD_LOCKSTEP", "1" if lockstep else "0")
    return run_device(qp, bs)


@pytest.mark.parametrize("op", ["gt", "lt"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_lockstep_equals_oracle_and_counts(hip_available, monkeypatch, case, op):
    qp, _ = compile_single_query(app(F2[op]))
    bs = batches(seed=len(case) + len(op), **CASES[case])
    ora = run_oracle(qp, bs)
    dev, c_ls, kind = run(qp, bs, monkeypatch, True)
    assert kind == 1 and len(ora[2]) > 0
    assert_same_rows(dev, ora)
    _, c_def, _ = run(qp, bs, monkeypatch, False)
    assert c_ls["partial_scans"] == c_def["partial_scans"]
    assert c_ls["matches"] == c_def["matches"] == len(ora[2])


def test_lockstep_null_e2_attributes(hip_available, monkeypatch):
    qp, _ = compile_single_query(app(F2["gt"], f1="price > 50"))
    bs = batches(nulls=True, seed=9, keys=2_000)
    ora = run_oracle(qp, bs)
    dev, _, _ = run(qp, bs, monkeypatch, True)
    assert len(ora[2]) > 0
    assert_same_rows(dev, ora)


def test_lockstep_time_going_back(hip_available, monkeypatch):
    qp, _ = compile_single_query(app(F2["gt"]))
    bs = batches(n=6_000, keys=300, delta=0.05, back=True, parts=2, seed=12)
    ora = run_oracle(qp, bs)
    dev, _, kind_ls = run(qp, bs, monkeypatch, True)
    _, _, kind_def = run(qp, bs, monkeypatch, False)
    assert kind_ls == kind_def
    assert_same_rows(dev, ora)


# f2 split per comparison (split_f2 / split_prep / split_eval): a comparison
# free of e2 decided once per partial, the e2 load on either side (swapped
# operators flipped), int / long e2 attributes converted to the comparison's
# type, the pre-resolved kinds (float column vs double: the StockStream
# configs; string equality; double) and the generic one, null e2 attributes
SPLIT_F2 = {
    "konst": "e1.volume > 20 and price > e1.price * 1.05",
    "konst-false": "e1.price < 0.0 and price > e1.price",
    "swapped": "e1.price * 0.97 > price",
    "cvt-long": "volume > e1.volume",
    "cvt-mixed": "volume > e1.price",
    "two-e2": "price > e1.price and volume < e1.volume",
    "ne": "price != e1.price and e1.price <= price",
}


@pytest.mark.parametrize("lockstep", [False, True])
@pytest.mark.parametrize("name", sorted(SPLIT_F2))
def test_split_f2_equals_oracle(hip_available, monkeypatch, name, lockstep):
    qp, _ = compile_single_query(app(SPLIT_F2[name]))
    bs = batches(nulls=True, seed=len(name), keys=2_000)
    ora = run_oracle(qp, bs)
    dev, c_split, kind = run(qp, bs, monkeypatch, lockstep)
    assert kind == 1
    assert_same_rows(dev, ora)
    monkeypatch.setenv("SHD_NO_SPLIT", "1")
    _, c_plain, _ = run(qp, bs, monkeypatch, lockstep)
    assert c_split["partial_scans"] == c_plain["partial_scans"]
    assert c_split["matches"] == c_plain["matches"] == len(ora[2])


def test_split_f2_float_int_schema(hip_available, monkeypatch):
    """The StockStream schema (float price, int volume): SK_F32_F64 (the
    configs' `price > e1.price * 1.05`) and SK_I32, against the oracle and the
    unsplit walk."""
    import numpy as np
    from siddhi_amd.runtime import ColumnBatch
    schema = "@app:playback define stream S (symbol string, price float, volume int); "
    q = (schema + "@info(name='q') from every e1=S[price > 60] -> e2=S[symbol == e1.symbol and "
         "price > e1.price * 1.05 and volume >= e1.volume] within 1 sec "
         "select e1.symbol as s, e1.price as p1, e2.price as p2, e2.volume as v insert into O;")
    qp, _ = compile_single_query(q)
    bs = []
    for o, b in batches(nulls=True, seed=31, keys=2_000):
        sym, price, vol = b.cols
        bs.append((o, ColumnBatch(b.ts, [sym, price.astype(np.float32), (vol % 1000).astype(np.int32)],
                                  b.nulls, b.call_offsets)))
    ora = run_oracle(qp, bs)
    for ls in (False, True):
        monkeypatch.delenv("SHD_NO_SPLIT", raising=False)
        dev, c_split, kind = run(qp, bs, monkeypatch, ls)
        assert kind == 1 and len(ora[2]) > 0
        assert_same_rows(dev, ora)
        monkeypatch.setenv("SHD_NO_SPLIT", "1")
        _, c_plain, _ = run(qp, bs, monkeypatch, ls)
        assert c_split["partial_scans"] == c_plain["partial_scans"]
        assert c_split["matches"] == c_plain["matches"] == len(ora[2])
