"""Multi-rank key routing (siddhi_amd/exchange.py) on the CPU with gloo,
world_size 2 and 4: round-robin input re-routed by key owner must give every rank
exactly the events of its keys in global arrival order, and the partitioned
pattern (config P3) evaluated per rank on the routed events must produce the
same matches as one engine over the whole stream."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from siddhi_amd import exchange as ex
from siddhi_amd import workloads as wl

N, KEYS, DELTA, CALL = 24000, 400, 0.05, 1024


def _rank_main(rank, world, path, outdir):
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    idx = np.arange(rank, N, world, dtype=np.int64)   # round-robin share of the global stream
    s, p, v, t = wl.stock_stream_at(idx, KEYS, DELTA, seed_offset=3)
    cols = [torch.from_numpy(s.astype(np.int32)), torch.from_numpy(p), torch.from_numpy(v), torch.from_numpy(t)]
    seq = torch.from_numpy(idx)
    # two micro-batches, each routed with one all-to-all
    parts = []
    half = len(idx) // 2
    for a, b in ((0, half), (half, len(idx))):
        rc, rseq, stats = ex.route([c[a:b] for c in cols], cols[0][a:b], seq[a:b], world)
        parts.append((rc, rseq))
    # null masks travel with their events (price null on every 7th, volume on every 5th global event)
    nul = [None, torch.from_numpy(idx % 7 == 0), torch.from_numpy(idx % 5 == 0), None]
    _, nseq, _, rn = ex.route(cols, cols[0], seq, world, nulls=nul)
    np.savez(os.path.join(outdir, "r%d.npz" % rank),
             **{"c%d_%d" % (i, j): parts[i][0][j].numpy() for i in range(2) for j in range(4)},
             seq0=parts[0][1].numpy(), seq1=parts[1][1].numpy(), nseq=nseq.numpy(),
             **{"n%d" % j: rn[j].numpy() for j in range(4)})
    dist.destroy_process_group()


@pytest.fixture(scope="module", params=[2, 4], ids=["world2", "world4"])
def routed(request, tmp_path_factory):
    world = request.param
    d = tmp_path_factory.mktemp("route")
    path = tempfile.mktemp(dir=str(d))
    mp.spawn(_rank_main, args=(world, path, str(d)), nprocs=world)
    return [np.load(os.path.join(str(d), "r%d.npz" % r)) for r in range(world)]


def test_route_delivers_own_keys_in_arrival_order(routed):
    s, p, v, t = wl.stock_stream(N, KEYS, DELTA, seed_offset=3)
    owner = ex.owner_of(torch.from_numpy(s.astype(np.int64)), len(routed)).numpy()
    for r, z in enumerate(routed):
        seq = np.concatenate([z["seq0"], z["seq1"]])
        want = np.nonzero(owner == r)[0]
        # micro-batch boundaries are global: batch 0 holds the first half of every rank's share
        assert np.array_equal(np.sort(seq), want)
        assert np.all(np.diff(z["seq0"]) > 0) and np.all(np.diff(z["seq1"]) > 0)
        sym = np.concatenate([z["c0_0"], z["c1_0"]]).astype(np.uint32)
        price = np.concatenate([z["c0_1"], z["c1_1"]])
        ts = np.concatenate([z["c0_3"], z["c1_3"]])
        assert np.array_equal(sym, s[seq]) and np.array_equal(price, p[seq]) and np.array_equal(ts, t[seq])


def test_route_carries_null_masks(routed):
    for r, z in enumerate(routed):
        seq = z["nseq"]
        assert np.all(np.diff(seq) > 0)
        assert not z["n0"].any() and not z["n3"].any()
        assert np.array_equal(z["n1"].astype(bool), seq % 7 == 0)
        assert np.array_equal(z["n2"].astype(bool), seq % 5 == 0)


def test_call_offsets_follow_global_calls():
    seq = torch.tensor([1, 5, 1023, 1024, 1030, 4096, 4097], dtype=torch.int64)
    assert ex.call_offsets_from_seq(seq, 1024).tolist() == [0, 3, 5, 7]


def test_partitioned_pattern_over_routed_ranks_matches_single_engine(routed):
    from parity import compile_single_query, run_oracle, stock_batch
    from siddhi_amd.runtime import ColumnBatch
    qp, _ = compile_single_query(wl.P3_APP)
    s, p, v, t = wl.stock_stream(N, KEYS, DELTA, seed_offset=3)
    whole = run_oracle(qp, [(0, stock_batch(s, p, v, t, CALL))])
    rows = []
    for z in routed:
        batches = []
        for i in range(2):
            seq = torch.from_numpy(z["seq%d" % i])
            offs = ex.call_offsets_from_seq(seq, CALL).numpy()
            cols = [z["c%d_0" % i].astype(np.uint32), z["c%d_1" % i], z["c%d_2" % i]]
            batches.append((0, ColumnBatch(z["c%d_3" % i], cols, [None] * 3, offs)))
        rows.append(run_oracle(qp, batches))
    assert len(whole[2]) > 0
    assert sum(len(r[2]) for r in rows) == len(whole[2])

    def canon(r):
        return sorted(zip(r[2].tolist(), r[3][:, 0].tolist(), r[3][:, 1].tolist(), r[3][:, 2].tolist()))
    merged = sorted(sum((canon(r) for r in rows), []))
    assert merged == canon(whole)


def _oracle_rows_with_seq(qp, batches):
    """Oracle per InputHandler call (as run_oracle) plus each row's in_seq."""
    from oracle_engine import OracleQueryEngine
    from parity import concat_rows
    from siddhi_amd.runtime import ColumnBatch
    eng = OracleQueryEngine(qp, None)
    parts, cid = [], 0
    for si, b in batches:
        offs = b.call_offsets
        for c in range(len(offs) - 1):
            s, e = int(offs[c]), int(offs[c + 1])
            sub = ColumnBatch(b.ts[s:e], [x[s:e] for x in b.cols], [None] * len(b.cols))
            for ch in eng.set_time(int(b.ts[e - 1])) + eng.push(si, sub):
                n = len(ch.ts)
                parts.append((np.full(n, cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                cid += 1
    seq = np.concatenate(eng.drained_seq) if eng.drained_seq else np.zeros(0, np.int64)
    eng.close()
    return concat_rows(parts), seq


def test_merged_rank_outputs_equal_single_engine_in_order(routed):
    """shd_out.in_seq-style merge (exchange.merge_outputs): the ranks' rows,
    each tagged with the global sequence of its emitting event, merge into
    exactly the rows, order and callback chunks of one engine over the whole
    stream."""
    from parity import assert_same_rows, compile_single_query, stock_batch
    from siddhi_amd.runtime import ColumnBatch
    qp, _ = compile_single_query(wl.P3_APP)
    s, p, v, t = wl.stock_stream(N, KEYS, DELTA, seed_offset=3)
    whole, wseq = _oracle_rows_with_seq(qp, [(0, stock_batch(s, p, v, t, CALL))])
    parts = []
    for z in routed:
        batches, gseq = [], []
        for i in range(2):
            seq = torch.from_numpy(z["seq%d" % i])
            offs = ex.call_offsets_from_seq(seq, CALL).numpy()
            cols = [z["c%d_0" % i].astype(np.uint32), z["c%d_1" % i], z["c%d_2" % i]]
            batches.append((0, ColumnBatch(z["c%d_3" % i], cols, [None] * 3, offs)))
            gseq.append(z["seq%d" % i])
        rows, lseq = _oracle_rows_with_seq(qp, batches)
        parts.append((rows, np.concatenate(gseq)[lseq]))   # rank-local arrival index -> global sequence
    merged = ex.merge_outputs(parts)
    assert len(whole[2]) > 0
    assert_same_rows(merged[:5], whole)
    assert np.array_equal(merged[5], wseq)
