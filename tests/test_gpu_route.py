"""HIP re-route passes (shd_route_bucket / shd_route_merge, csrc/route.hip) on one
GPU: `world` senders are simulated in one process, the all-to-all is emulated by
slicing the send buffers, and the result must equal the torch reference
routing of exchange.route (owner bucket + stable sort by sequence) bit for bit,
with the call boundaries of exchange.call_offsets_from_seq."""
import numpy as np
import pytest
import torch

from siddhi_amd import exchange as ex

pytestmark = pytest.mark.gpu


def _stream(n_local, world, keys, seed, dev):
    g = torch.Generator().manual_seed(seed)
    out = []
    for r in range(world):
        seq = torch.arange(n_local, dtype=torch.int64) * world + r
        sym = torch.randint(0, keys, (n_local,), generator=g, dtype=torch.int32)
        price = torch.rand(n_local, generator=g, dtype=torch.float64) * 100
        vol = torch.randint(-2 ** 40, 2 ** 40, (n_local,), generator=g, dtype=torch.int64)
        ts = 1_700_000_000_000 + seq // 7
        out.append([c.to(dev) for c in (sym, price, vol, ts, seq)])
    return out


def _check_route(world, n_local, a, b, keys=1000, call=1024, seed=1):
    dev = torch.device("cuda", 0)
    ranks = _stream(n_local, world, keys, seed, dev)
    lo = (a * world) // call * call
    nblocks = -(-(b * world - lo) // call)
    sends = []
    for sym, price, vol, ts, seq in ranks:
        cols = [sym[a:b].contiguous(), price[a:b].contiguous(), vol[a:b].contiguous(), ts[a:b].contiguous()]
        send, counts, words = ex.bucket(cols, sym[a:b].contiguous(), seq[a:b].contiguous(), world, lo)
        sends.append((send.view(-1, words), counts.cpu().tolist()))
        # stable buckets: owner-major, batch order inside each owner
        own = ex.owner_of(sym[a:b], world)
        order = torch.sort(own.to(torch.uint8), stable=True)[1]
        seqoff = (send.view(-1, words)[:, words - 1] >> 32) if words else None
        assert torch.equal(seqoff, seq[a:b][order] - lo)
        assert counts.cpu().tolist() == torch.bincount(own, minlength=world).cpu().tolist()
    for d in range(world):
        parts, rc = [], []
        for s in range(world):
            send, cnt = sends[s]
            off = sum(cnt[:d])
            parts.append(send[off:off + cnt[d]])
            rc.append(cnt[d])
        recv = torch.cat(parts).reshape(-1).contiguous()
        outs, rseq, co = ex.merge(recv, torch.tensor(rc, dtype=torch.int64, device=dev),
                                  [torch.int32, torch.float64, torch.int64, torch.int64], world, lo, call, nblocks)
        # torch reference: every rank's rows owned by d, in sequence order
        allc = [torch.cat([r[j][a:b] for r in ranks]) for j in range(5)]
        mask = ex.owner_of(allc[0], world) == d
        o = torch.sort(allc[4][mask], stable=True)[1]
        ref = [c[mask][o] for c in allc]
        assert torch.equal(rseq, ref[4])
        for got, want in zip(outs, ref[:4]):
            assert torch.equal(got, want)
        want_co = ex.call_offsets_from_seq(ref[4], call).numpy() if ref[4].numel() else np.zeros(1, np.int64)
        assert np.array_equal(co, want_co), (co[:8], want_co[:8])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_route_matches_torch_reference(world):
    _check_route(world, 70_001, 0, 70_001)


def test_route_mid_stream_micro_batch_and_ragged_calls():
    # a micro-batch that starts and ends inside calls of the global stream
    _check_route(4, 50_000, 12_345, 41_000, call=1000)


def test_route_busy_keys_and_small_calls():
    _check_route(5, 20_000, 0, 20_000, keys=3, call=7)


def test_route_empty_and_tiny_batches():
    _check_route(2, 10, 3, 3)
    _check_route(8, 5, 0, 5)


def test_route_rejects_rows_outside_the_calls():
    dev = torch.device("cuda", 0)
    sym = torch.arange(100, dtype=torch.int32, device=dev)
    seq = torch.arange(100, dtype=torch.int64, device=dev)
    send, counts, words = ex.bucket([sym], sym, seq, 1, 0)
    with pytest.raises(ValueError):
        ex.merge(send, counts, [torch.int32], 1, 0, 10, 5)   # calls cover seq 0..49 only
