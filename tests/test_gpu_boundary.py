"""SURVEY.md §8b boundary fields through the C-ABI on the device:
shd_out.state_idx (the state whose processor emitted a row) and
shd_batch.base_seq (global arrival index of a batch's first event, so that
shd_out.in_seq is global on a key-sharded rank)."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, concat_rows, run_oracle, stock_batch
from siddhi_amd import workloads as wl

pytestmark = pytest.mark.gpu


def _push_all(qp, batches, base=None):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    dq = DeviceQuery(qp.ir)
    parts, seqs, sidx = [], [], []
    try:
        for j, (si, b) in enumerate(batches):
            cols = [np.ascontiguousarray(c) for c in b.cols]
            t = np.ascontiguousarray(b.ts, np.int64)
            dq.push_raw(si, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0] * len(cols), SHD_MEM_HOST,
                        b.call_offsets, True, base_seq=None if base is None else base[j])
            r = dq.poll(with_seq=True)
            if r is not None:
                parts.append(r[:5])
                seqs.append(r[5])
                sidx.append(dq.last_state_idx)
        kind = dq.engine_kind
    finally:
        dq.close()
    cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64)
    return concat_rows(parts), cat(seqs), cat(sidx), kind


def _batches(n, keys, delta, seed, cuts):
    sym, price, vol, ts = wl.stock_stream(n, keys, delta, seed_offset=seed)
    return [(0, stock_batch(sym[a:b], price[a:b], vol[a:b], ts[a:b], 500)) for a, b in zip(cuts[:-1], cuts[1:])]


def test_base_seq_makes_in_seq_global(hip_available):
    """Two pushes that are a rank's share of a longer stream: with base_seq
    the rows' in_seq are the global arrival indices (local index + base)."""
    qp, _ = compile_single_query(wl.P3_APP)
    batches = _batches(20_000, 500, 0.05, 3, [0, 9000, 20_000])
    dev0, seq0, _, _ = _push_all(qp, batches)
    dev1, seq1, _, _ = _push_all(qp, batches, base=[1_000_000, 5_000_000])
    assert len(seq0) > 0
    assert_same_rows(dev1, dev0)
    glob = np.where(seq0 < 9000, seq0 + 1_000_000, seq0 - 9000 + 5_000_000)
    np.testing.assert_array_equal(seq1, glob)


def test_base_seq_must_not_go_back(hip_available):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST, SiddhiHipError, SHD_E_ARG
    qp, _ = compile_single_query(wl.P3_APP)
    (_, b), = _batches(2000, 50, 0.05, 4, [0, 2000])
    dq = DeviceQuery(qp.ir)
    try:
        cols = [np.ascontiguousarray(c) for c in b.cols]
        t = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(0, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0] * 3, SHD_MEM_HOST, None, True,
                    base_seq=10_000)
        with pytest.raises(SiddhiHipError) as ei:
            dq.push_raw(0, b.n, t.ctypes.data, [c.ctypes.data for c in cols], [0] * 3, SHD_MEM_HOST, None, True,
                        base_seq=10_500)
        assert ei.value.code == SHD_E_ARG
    finally:
        dq.close()


@pytest.mark.parametrize("name,app,expect", [
    ("P3", wl.P3_APP, {1}),
    ("S4-or", wl.S4_APPS["or"], {1, 2}),
    ("S4-seq", wl.S4_APPS["seqplus"], {2}),
    ("W2", wl.W2_LENGTH_APP, {0}),
], ids=lambda x: x if isinstance(x, str) else "")
def test_state_idx_names_the_emitting_state(hip_available, name, app, expect):
    qp, _ = compile_single_query(app)
    batches = _batches(30_000, 300 if name == "P3" else 40, 0.5, 6, [0, 14_000, 30_000])
    ora = run_oracle(qp, batches)
    dev, _, sidx, _ = _push_all(qp, batches)
    assert len(ora[2]) > 0
    assert set(np.unique(sidx).tolist()) <= expect
    if name == "S4-or":
        # the reference numbers a logical state's operands second-first
        # (StateInputStreamParser.java:349-361): e3 is state 1, e2 state 2;
        # rows completed by e2 carry p2 (p3 null), rows completed by e3 carry p3
        p3_null = dev[4][:, 2].astype(bool)
        np.testing.assert_array_equal(sidx, np.where(p3_null, 2, 1))
        assert set(np.unique(sidx).tolist()) == {1, 2}
