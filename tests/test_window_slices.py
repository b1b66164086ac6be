"""Time-sliced window aggregates over ranks (siddhi_amd/exchange.py: window_of,
exchange_tail, halo_covers, halo_take) on the CPU with gloo, world_size 2 and
3: every rank takes one contiguous slice of the global stream, receives the
tail of the previous rank's slice (the halo) point-to-point, pushes it through
a fresh query whose rows it drops, then its own slice.  The ranks' rows,
concatenated in rank order, must equal one query over the whole stream (same
InputHandler calls): row count, types, timestamps, group keys, counts and
callback chunks exactly, double aggregates within 1e-9 relative (the halo
query's running sums have a different history).  The per-rank query here is
the CPU oracle; tests/test_gpu_window_slices.py runs the device query.

Reference: LengthWindowProcessor.process (C/query/processor/stream/window/
LengthWindowProcessor.java:106-142), TimeWindowProcessor expiry
(TimeWindowProcessor.java:144-145)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from siddhi_amd import exchange as ex
from siddhi_amd import workloads as wl

N, KEYS, DELTA, CALL = 8192, 40, 0.05, 1024
APPS = {
    "length": ("@app:playback " + wl.STOCK_DEF + " @info(name='q') from StockStream[price>60]#window.length(3000) "
               "select symbol, sum(price) as s, avg(volume) as a, count() as c group by symbol insert into O;"),
    "time": ("@app:playback " + wl.STOCK_DEF + " @info(name='q') from StockStream[price>60]#window.time(200 millisec) "
             "select symbol, sum(price) as s, avg(price) as m, count() as c group by symbol insert into O;"),
}


def slice_columns(rank):
    return wl.stock_stream(N, KEYS, DELTA, seed_offset=5, start=rank * N)


def oracle_after_halo(qp, halo, own):
    """Oracle rows of `own` (calls of CALL events) after the halo's calls, whose
    rows are dropped; chunk ids count from 0 at `own`."""
    from oracle_engine import OracleQueryEngine
    from parity import concat_rows
    from siddhi_amd.runtime import ColumnBatch
    eng = OracleQueryEngine(qp, None)
    parts, cid = [], 0
    for keep, cols in ((False, halo), (True, own)):
        if cols is None:
            continue
        s, p, v, t = cols
        for a in range(0, len(t), CALL):
            b = min(len(t), a + CALL)
            sub = ColumnBatch(t[a:b], [s[a:b], p[a:b], v[a:b]], [None] * 3)
            for ch in eng.set_time(int(t[b - 1])) + eng.push(0, sub):
                if keep:
                    parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                    cid += 1
    eng.close()
    return concat_rows(parts)


def _rank_main(rank, world, path, outdir, kind):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from parity import compile_single_query
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    qp, _ = compile_single_query(APPS[kind])
    window = ex.window_of(qp)
    s, p, v, t = slice_columns(rank)
    cols = [torch.from_numpy(s.astype(np.int32)), torch.from_numpy(p), torch.from_numpy(v), torch.from_numpy(t)]

    def prime(halo):
        hp, ht = halo[1].numpy(), halo[3]
        carry = min(window[1], int((hp > 60.0).sum())) if window[0] == "length" else 0
        return ex.halo_covers(window, carry, ht, int(t[0]))

    take = ex.halo_take(window, N, lambda k: ex.exchange_tail(cols, k, rank, world), prime)
    halo = ex.exchange_tail(cols, take, rank, world)
    hc = None if halo is None else (halo[0].numpy().astype(np.uint32), halo[1].numpy(), halo[2].numpy(),
                                    halo[3].numpy())
    rows = oracle_after_halo(qp, hc, (s, p, v, t))
    np.savez(os.path.join(outdir, "%s_w%d_r%d.npz" % (kind, world, rank)), take=take,
             **{"x%d" % i: a for i, a in enumerate(rows)})
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["length", "time"])
def test_sliced_window_rows_equal_one_query(tmp_path, world, kind):
    from parity import assert_rows_agg, compile_single_query, run_oracle, stock_batch
    path = tempfile.mktemp(dir=str(tmp_path))
    mp.spawn(_rank_main, args=(world, path, str(tmp_path), kind), nprocs=world)
    qp, _ = compile_single_query(APPS[kind])
    whole = run_oracle(qp, [(0, stock_batch(*slice_columns(r), CALL)) for r in range(world)])
    parts, base = [], 0
    for r in range(world):
        z = np.load(os.path.join(str(tmp_path), "%s_w%d_r%d.npz" % (kind, world, r)))
        x = [z["x%d" % i] for i in range(5)]
        if r > 0:
            take = int(z["take"])
            assert 0 < take <= N
        x[0] = x[0] + base
        base = int(x[0].max()) + 1 if len(x[0]) else base
        parts.append(tuple(x))
    merged = tuple(np.concatenate([q[i] for q in parts]) for i in range(5))
    assert len(whole[2]) > 0
    assert_rows_agg(merged, whole, qp, exact=False)


def test_halo_covers_rules():
    ts = torch.tensor([100, 101, 105, 130], dtype=torch.int64)
    assert ex.halo_covers(("length", 5), 5, ts, 131)
    assert not ex.halo_covers(("length", 5), 4, ts, 131)
    assert ex.halo_covers(("time", 30), 0, ts, 131)        # 100 + 30 < 131
    assert not ex.halo_covers(("time", 31), 0, ts, 131)
    assert not ex.halo_covers(("time", 10), 0, ts[[0, 2, 1, 3]], 200)   # timestamps going back
    assert not ex.halo_covers(("time", 10), 0, ts[:0], 200)


def test_window_of_reads_the_plan():
    from parity import compile_single_query
    assert ex.window_of(compile_single_query(APPS["length"])[0]) == ("length", 3000)
    assert ex.window_of(compile_single_query(APPS["time"])[0]) == ("time", 200)
    assert ex.window_of(compile_single_query(wl.P3_APP)[0]) is None


def _rank_too_long(rank, world, path, outdir):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    n = 500
    cols = [torch.arange(n, dtype=torch.int64) + rank * n]
    # a length window of 2000 filter-passing items cannot be covered by a 500-event slice
    try:
        ex.halo_take(("length", 2000), n, lambda k: ex.exchange_tail(cols, k, rank, world),
                     lambda halo: halo[0].numel() >= 2000)
        ok = "returned"
    except ValueError:
        ok = "raised"
    with open(os.path.join(outdir, "too_long_r%d.txt" % rank), "w") as f:
        f.write(ok)
    dist.destroy_process_group()


def test_halo_take_raises_past_a_whole_slice(tmp_path):
    """Every rank learns the same outcome: a window reaching past the whole
    previous slice raises on all ranks (the flag is all-reduced)."""
    path = tempfile.mktemp(dir=str(tmp_path))
    mp.spawn(_rank_too_long, args=(2, path, str(tmp_path)), nprocs=2)
    for r in range(2):
        assert open(os.path.join(str(tmp_path), "too_long_r%d.txt" % r)).read() == "raised"


def test_exchange_tail_is_a_no_op_alone():
    cols = [torch.arange(10)]
    assert ex.exchange_tail(cols, 4, 0, 1) is None
    assert ex.exchange_tail(cols, 0, 0, 2) is None


SLICE_LENS = [8192, 5120, 6144]   # a stream that does not divide evenly over 3 ranks


def slice_columns_nulls(rank):
    """Slice `rank` of one global stream with ~5% null prices; slices of
    unequal length (SLICE_LENS), cut on calls."""
    n = SLICE_LENS[rank]
    start = sum(SLICE_LENS[:rank])
    s, p, v, t = wl.stock_stream(sum(SLICE_LENS), KEYS, DELTA, seed_offset=6)
    s, p, v, t = s[start:start + n], p[start:start + n], v[start:start + n], t[start:start + n]
    rng = np.random.default_rng(1000 + rank)
    null = (rng.random(n) < 0.05).astype(np.uint8)
    return s, p, v, t, null


def oracle_after_halo_nulls(qp, halo, own):
    from oracle_engine import OracleQueryEngine
    from parity import concat_rows
    from siddhi_amd.runtime import ColumnBatch
    eng = OracleQueryEngine(qp, None)
    parts, cid = [], 0
    for keep, cols in ((False, halo), (True, own)):
        if cols is None:
            continue
        s, p, v, t, nl = cols
        for a in range(0, len(t), CALL):
            b = min(len(t), a + CALL)
            sub = ColumnBatch(t[a:b], [s[a:b], p[a:b], v[a:b]], [None, nl[a:b], None])
            for ch in eng.set_time(int(t[b - 1])) + eng.push(0, sub):
                if keep:
                    parts.append((np.full(len(ch.ts), cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                    cid += 1
    eng.close()
    return concat_rows(parts)


def _rank_nulls(rank, world, path, outdir, kind):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from parity import compile_single_query
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    qp, _ = compile_single_query(APPS[kind])
    window = ex.window_of(qp)
    s, p, v, t, nl = slice_columns_nulls(rank)
    cols = [torch.from_numpy(s.astype(np.int32)), torch.from_numpy(p), torch.from_numpy(v), torch.from_numpy(t)]
    nulls = [None, torch.from_numpy(nl), None, None]

    def prime(halo):
        (hs, hp, hv, ht), hn = halo
        passing = (hp.numpy() > 60.0) & (hn[1].numpy() == 0)   # a null price fails `price > 60`
        carry = min(window[1], int(passing.sum())) if window[0] == "length" else 0
        return ex.halo_covers(window, carry, ht, int(t[0]))

    take = ex.halo_take(window, len(t), lambda k: ex.exchange_tail(cols, k, rank, world, nulls=nulls), prime)
    halo = ex.exchange_tail(cols, take, rank, world, nulls=nulls)
    hc = None
    if halo is not None:
        (hs, hp, hv, ht), hn = halo
        hc = (hs.numpy().astype(np.uint32), hp.numpy(), hv.numpy(), ht.numpy(), hn[1].numpy())
    rows = oracle_after_halo_nulls(qp, hc, (s, p, v, t, nl))
    np.savez(os.path.join(outdir, "n%s_w%d_r%d.npz" % (kind, world, rank)), take=take,
             **{"x%d" % i: a for i, a in enumerate(rows)})
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["length", "time"])
def test_sliced_window_nulls_unequal_slices(tmp_path, kind):
    """the halo carries the null masks (a null price primes the
    query as null), and slices of unequal length agree on one halo size (the
    shortest slice bounds it on every rank); world 3, rows == one query."""
    from parity import assert_rows_agg, compile_single_query, run_oracle
    from siddhi_amd.runtime import ColumnBatch
    world = 3
    path = tempfile.mktemp(dir=str(tmp_path))
    mp.spawn(_rank_nulls, args=(world, path, str(tmp_path), kind), nprocs=world)
    qp, _ = compile_single_query(APPS[kind])
    batches = []
    for r in range(world):
        s, p, v, t, nl = slice_columns_nulls(r)
        offs = np.append(np.arange(0, len(t), CALL, dtype=np.int64), np.int64(len(t)))
        batches.append((0, ColumnBatch(t, [s, p, v], [None, nl, None], offs)))
    whole = run_oracle(qp, batches)
    parts, base = [], 0
    for r in range(world):
        z = np.load(os.path.join(str(tmp_path), "n%s_w%d_r%d.npz" % (kind, world, r)))
        x = [z["x%d" % i] for i in range(5)]
        x[0] = x[0] + base
        base = int(x[0].max()) + 1 if len(x[0]) else base
        parts.append(tuple(x))
    merged = tuple(np.concatenate([q[i] for q in parts]) for i in range(5))
    assert len(whole[2]) > 0
    assert_rows_agg(merged, whole, qp, exact=False)
