"""Key-sharded P3 on the device: the stream's events split by
key owner (exchange.owner_of) over two device queries standing in for two
ranks; each rank's rows carry shd_out.in_seq, mapped to the global sequence
and k-way merged (exchange.merge_outputs).  The merged rows -- order, values,
timestamps and callback chunks -- must equal one device query over the whole
stream and the CPU oracle.  Also: in_seq of every engine equals the oracle's."""
import os

import numpy as np
import pytest
import torch

from parity import assert_same_rows, compile_single_query, concat_rows, run_oracle, stock_batch
from siddhi_amd import exchange as ex
from siddhi_amd import workloads as wl
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu


def _device_rows_with_seq(qp, batches):
    from siddhi_amd.hip_engine import DeviceQuery, SHD_MEM_HOST
    dq = DeviceQuery(qp.ir)
    parts, seqs = [], []
    for si, b in batches:
        cols = [np.ascontiguousarray(c) for c in b.cols]
        ts = np.ascontiguousarray(b.ts, np.int64)
        dq.push_raw(si, b.n, ts.ctypes.data, [c.ctypes.data for c in cols], [0] * len(cols), SHD_MEM_HOST,
                    b.call_offsets if len(b.call_offsets) > 2 else None, True)
        r = dq.poll(with_seq=True)
        if r is not None:
            parts.append(r[:5])
            seqs.append(r[5])
    dq.close()
    return concat_rows(parts), (np.concatenate(seqs) if seqs else np.zeros(0, np.int64))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_p3_merges_to_single_engine_order(hip_available, world):
    qp, _ = compile_single_query(wl.P3_APP)
    n, keys, call = 120_000, 3000, 1024
    s, p, v, t = wl.stock_stream(n, keys, 0.02, seed_offset=19)
    whole = run_oracle(qp, [(0, stock_batch(s, p, v, t, call))])
    one, _ = _device_rows_with_seq(qp, [(0, stock_batch(s, p, v, t, call))])
    assert len(whole[2]) > 0
    assert_same_rows(one, whole)
    owner = ex.owner_of(torch.from_numpy(s.astype(np.int64)), world).numpy()
    parts = []
    for r in range(world):
        gseq = np.nonzero(owner == r)[0]          # this rank's events in global arrival order
        offs = ex.call_offsets_from_seq(torch.from_numpy(gseq), call).numpy()
        cut = int(offs[len(offs) // 2])            # two micro-batches per rank, cut at a call boundary
        batches = []
        for a, b in ((0, cut), (cut, len(gseq))):
            if b <= a:
                continue
            idx = gseq[a:b]
            o = ex.call_offsets_from_seq(torch.from_numpy(idx), call).numpy()
            batches.append((0, ColumnBatch(t[idx], [s[idx], p[idx], v[idx]], [None] * 3, o)))
        rows, lseq = _device_rows_with_seq(qp, batches)
        parts.append((rows, gseq[lseq]))
    merged = ex.merge_outputs(parts)
    assert_same_rows(merged[:5], whole)


CASES = [("P3", wl.P3_APP, 60_000, 2000, 0.02), ("W2-length", wl.W2_LENGTH_APP, 40_000, 300, 0.1),
         ("S4-seqplus", wl.S4_APPS["seqplus"], 8_000, 100, 1.0), ("S4-not", wl.S4_APPS["not"], 8_000, 100, 1.0)]


@pytest.mark.parametrize("name,app,n,keys,delta", CASES, ids=[c[0] for c in CASES])
def test_in_seq_equals_oracle(hip_available, name, app, n, keys, delta):
    """shd_out.in_seq (the emitting event's arrival index) on every engine."""
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from test_exchange import _oracle_rows_with_seq
    qp, _ = compile_single_query(app)
    s, p, v, t = wl.stock_stream(n, keys, delta, seed_offset=23)
    batches = [(0, stock_batch(s[a:b], p[a:b], v[a:b], t[a:b], 512)) for a, b in ((0, n // 2), (n // 2, n))]
    ora, oseq = _oracle_rows_with_seq(qp, batches)
    dev, dseq = _device_rows_with_seq(qp, batches)
    assert len(ora[2]) > 0
    assert len(dseq) == len(oseq)
    assert np.array_equal(dseq, oseq)


N_RR, KEYS_RR, DELTA_RR, BATCH_RR = 200_000, 4000, 0.02, 30_720


def _rr_rank(rank, world, path, outdir, staged):
    """One rank of the N > 1 bench path on a shared GPU: its round-robin share
    of the global stream resident in HBM, each micro-batch re-routed by key
    owner with the HIP bucket / merge passes (the all-to-all staged through host
    tensors over gloo), pushed to this rank's P3 query."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for q in (root, os.path.join(root, "tests")):
        if q not in sys.path:
            sys.path.insert(0, q)
    import torch.distributed as dist
    from siddhi_amd import exchange as ex2
    from siddhi_amd import hip_engine as he
    from siddhi_amd import workloads as wl2
    from parity import compile_single_query as csq
    dist.init_process_group("gloo", init_method="file://" + path, rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    qp, _ = csq(wl2.P3_APP)
    idx = np.arange(rank, N_RR, world, dtype=np.int64)
    s, p, v, t = wl2.stock_stream_at(idx, KEYS_RR, DELTA_RR, seed_offset=0)
    cols = [torch.from_numpy(s.astype(np.int32)).to(dev), torch.from_numpy(p).to(dev),
            torch.from_numpy(v).to(dev), torch.from_numpy(t).to(dev)]
    seq = torch.from_numpy(idx).to(dev)
    dq = he.DeviceQuery(qp.ir)
    parts, lseqs, routed = [], [], []

    def job(a, b):
        lo = (a * world) // 1024 * 1024
        nb = -(-(b * world - lo) // 1024)
        if not staged:
            return lambda: ex2.route_device([c[a:b] for c in cols], cols[0][a:b], seq[a:b], world, lo, 1024, nb,
                                            stage_host=True)
        return (lambda: ex2.route_stage_a([c[a:b] for c in cols], cols[0][a:b], seq[a:b], world, lo,
                                          stage_host=True),
                lambda st: ex2.route_stage_b(st, 1024, nb))

    cuts = list(range(0, len(idx), BATCH_RR)) + [len(idx)]   # BATCH_RR * world: whole 1024-event calls
    pipe = ex2.RoutePipeline(0)   # micro-batch k+1 routed while k is pushed (bench.py's N > 1 path)
    jobs = [job(a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    engine_stream = torch.cuda.ExternalStream(dq.stream_handle(), device=dev)
    held = None
    for res in (pipe.run_staged(jobs) if staged else pipe.run(jobs)):
        (rs, rp, rv, rt), rseq, co, _ = res
        m = rs.numel()
        if m == 0:
            continue
        if staged:
            engine_stream.wait_event(co.event)   # the merge done before the engine reads its rows
            co = co.get()
        dq.push_raw(0, m, rt.data_ptr(), [rs.data_ptr(), rp.data_ptr(), rv.data_ptr()], [0, 0, 0],
                    he.SHD_MEM_DEVICE, co.astype(np.int64), True)
        held = res   # RoutePipeline lifetime: kept until the next push has returned
        routed.append(rseq.cpu().numpy())
        r = dq.poll(with_seq=True)
        if r is not None:
            parts.append(r[:5])
            lseqs.append(r[5])
    pipe.close()
    dq.close()
    gall = np.concatenate(routed) if routed else np.zeros(0, np.int64)
    rows = concat_rows(parts)
    lseq = np.concatenate(lseqs) if lseqs else np.zeros(0, np.int64)
    np.savez(os.path.join(outdir, "r%d.npz" % rank), c=rows[0], ty=rows[1], ts=rows[2], v=rows[3], n=rows[4],
             g=gall[lseq] if len(lseq) else np.zeros(0, np.int64))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,staged", [(2, False), (4, False), (2, True), (4, True)])
def test_roundrobin_route_device_merges_to_single_engine(hip_available, tmp_path, world, staged):
    """The N > 1 bench path end to end (bench.py --input roundrobin): 2 or 4
    ranks on one GPU, HIP bucket -> all-to-all -> HIP merge -> P3 query per rank,
    the next micro-batch routed while the current one is pushed
    (exchange.RoutePipeline; staged: run_staged -- counts exchanged one
    micro-batch ahead through pinned host copies, the merge fenced by an
    event on the engine's stream), rows mapped to global sequence numbers and
    k-way merged (exchange.merge_outputs): equal to one device query over the
    whole stream and to the CPU oracle."""
    import tempfile
    import torch.multiprocessing as mp
    mp.spawn(_rr_rank, args=(world, tempfile.mktemp(dir=str(tmp_path)), str(tmp_path), staged), nprocs=world)
    parts = []
    for r in range(world):
        z = np.load(os.path.join(str(tmp_path), "r%d.npz" % r))
        parts.append(((z["c"], z["ty"], z["ts"], z["v"], z["n"]), z["g"]))
    merged = ex.merge_outputs(parts)
    qp, _ = compile_single_query(wl.P3_APP)
    s, p, v, t = wl.stock_stream_at(np.arange(N_RR, dtype=np.int64), KEYS_RR, DELTA_RR, seed_offset=0)
    whole = run_oracle(qp, [(0, stock_batch(s, p, v, t, 1024))])
    one, _ = _device_rows_with_seq(qp, [(0, stock_batch(s, p, v, t, 1024))])
    assert len(whole[2]) > 50
    assert_same_rows(one, whole)
    assert merged is not None
    assert_same_rows(merged[:5], whole)
