"""Key-hash routing of micro-batches across GPUs.

A partitioned query keeps all of its state per partition key
(PartitionStateHolder.getState, modules/siddhi-core/src/main/java/io/siddhi/
core/util/snapshot/state/PartitionStateHolder.java:43-48; per-key seeding in
PartitionStreamReceiver.send, .../partition/PartitionStreamReceiver.java:262-283),
so keys are sharded over ranks: owner(key) = hash32(key) % world.  Input that
arrives pre-partitioned is pushed by its owner directly.  Input that does not
is re-routed with ONE all-to-all per micro-batch (torch.distributed: backend
"nccl" is RCCL over xGMI on MI355X, "gloo" in the CPU tests): every rank
buckets its events by owner, exchanges bucket sizes, then the packed event
rows; the receiver restores global arrival order with a stable sort on the
event sequence number.  Per key this reproduces exactly the event order and
InputHandler-call membership the reference sees, which is all a partitioned
query's output depends on.

Columns travel as one packed int64 matrix (one collective for all columns):
int32 / uint32 ids widen to int64, float64 travels as its bit pattern.

On the GPU (`route_device`) both local passes are HIP kernels behind the
C-ABI (`shd_route_bucket` / `shd_route_merge`, siddhi_amd/csrc/route.hip): a
stable bucket-by-owner scatter straight into the packed send buffer, and a
merge that puts the received rows back into global arrival order one
InputHandler call per workgroup (no sort), unpacking the columns and yielding
the call boundaries on the way.  4-byte columns and the sequence number travel
as 4-byte halves of a word (P3: 32 bytes per event instead of 40).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

_M32 = 0xFFFFFFFF


def hash32(keys: torch.Tensor) -> torch.Tensor:
    """Murmur3 fmix32 of the low 32 bits of integer keys (dictionary ids)."""
    x = keys.to(torch.int64) & _M32
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & _M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & _M32
    x = x ^ (x >> 16)
    return x


def owner_of(keys: torch.Tensor, world: int) -> torch.Tensor:
    return hash32(keys) % world


def pack(cols: List[torch.Tensor]) -> torch.Tensor:
    """[n, k] int64 matrix; float64 columns by bit pattern, int columns widened."""
    out = []
    for c in cols:
        if c.dtype == torch.float64:
            out.append(c.view(torch.int64))
        elif c.dtype == torch.float32:
            out.append(c.view(torch.int32).to(torch.int64))
        else:
            out.append(c.to(torch.int64))
    return torch.stack(out, dim=1).contiguous()


def unpack(m: torch.Tensor, dtypes: List[torch.dtype]) -> List[torch.Tensor]:
    cols = []
    for j, dt in enumerate(dtypes):
        c = m[:, j].contiguous()
        if dt == torch.float64:
            cols.append(c.view(torch.float64))
        elif dt == torch.float32:
            cols.append(c.to(torch.int32).view(torch.float32))
        else:
            cols.append(c.to(dt))
    return cols


def route(cols: List[torch.Tensor], key: torch.Tensor, seq: torch.Tensor, world: int,
          group: Optional[dist.ProcessGroup] = None, nulls: Optional[List[Optional[torch.Tensor]]] = None):
    """All-to-all re-route of one micro-batch by key owner.

    cols:  the event columns (1-D, equal length, any of int32/int64/float64);
    key:   the partition key of every event (integer ids);
    seq:   global arrival sequence numbers (int64);
    nulls: optional per-column null masks (bool/uint8, None = no nulls); they
           travel as one extra packed bit-mask column.
    Returns (received columns, received seq, stats), in increasing seq order,
    plus the received null masks (uint8, one per column) when `nulls` is given.
    """
    if nulls is not None:
        if len(nulls) != len(cols) or len(cols) > 62:
            raise ValueError("one null mask (or None) per column, at most 62 columns")
        bits = torch.zeros(seq.numel(), dtype=torch.int64, device=seq.device)
        for j, m in enumerate(nulls):
            if m is not None:
                bits |= m.to(torch.int64) << j
        rc, rseq, stats = route(list(cols) + [bits], key, seq, world, group)
        rb = rc.pop()
        return rc, rseq, stats, [((rb >> j) & 1).to(torch.uint8) for j in range(len(cols))]
    dtypes = [c.dtype for c in cols]
    if world == 1:
        order = _seq_order(seq)
        return [c[order] for c in cols], seq[order], {"sent": 0, "received": 0}
    if world > 256:
        raise ValueError("route: world %d > 256 (owners are bucketed with one 8-bit pass)" % world)
    owner = owner_of(key, world)
    # stable bucket order by owner: one 8-bit radix pass (world <= 256)
    _, order = torch.sort(owner.to(torch.uint8), stable=True)
    send = pack([c[order] for c in cols] + [seq[order]])
    counts = torch.bincount(owner, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts, group=group)
    k = send.shape[1]
    in_splits = (counts * k).tolist()
    out_splits = (recv_counts * k).tolist()
    recv = torch.empty(int(sum(out_splits)), dtype=torch.int64, device=send.device)
    dist.all_to_all_single(recv, send.reshape(-1), out_splits, in_splits, group=group)
    recv = recv.view(-1, k)
    # every sender's rows arrive in seq order; restore the global order
    o = _seq_order(recv[:, k - 1])
    out = [c[o] for c in unpack(recv[:, :k - 1], dtypes)]
    rseq = recv[:, k - 1][o]
    rank = dist.get_rank(group)
    stats = {"sent": int(counts.sum().item() - counts[rank].item()),
             "received": int(recv_counts.sum().item() - recv_counts[rank].item())}
    return out, rseq, stats


def _seq_order(seq: torch.Tensor) -> torch.Tensor:
    """Stable ascending order of sequence numbers; sorted on 32-bit offsets from
    the minimum when the micro-batch's span fits (half the radix passes)."""
    if seq.numel() == 0:
        return torch.zeros(0, dtype=torch.int64, device=seq.device)
    lo = seq.min()
    if int(seq.max() - lo) < 2 ** 31:
        _, o = torch.sort((seq - lo).to(torch.int32), stable=True)
    else:
        _, o = torch.sort(seq, stable=True)
    return o


def merge_outputs(parts):
    """k-way merge of key-sharded query outputs into the single-engine order.

    parts: per rank (rows, global_seq) where rows = (chunk, type, ts, values,
    nulls) as polled from the rank's query (DeviceQuery.poll) and global_seq[i]
    is the global arrival sequence of the input event that emitted row i (the
    rank's routed `seq` indexed by shd_out.in_seq).  A partitioned query's
    output for one input event comes from the rank owning its key, and each
    rank's rows are in (event, processor, pending-list) order, so a stable
    merge on the global sequence reproduces the order one engine over the
    whole stream emits (MultiProcessStreamReceiver: one callback chunk per
    (event, processor), C/query/input/MultiProcessStreamReceiver.java:94-124).
    Chunk ids are renumbered: a new chunk starts where the rank or the rank's
    chunk id changes.  Returns the merged (chunk, type, ts, values, nulls, seq).
    """
    import numpy as np
    live = [(r, rows, np.asarray(g, np.int64)) for r, (rows, g) in enumerate(parts) if rows is not None and len(g)]
    if not live:
        return None
    seq = np.concatenate([g for _, _, g in live])
    rank = np.concatenate([np.full(len(g), r, np.int64) for r, _, g in live])
    local = np.concatenate([np.arange(len(g), dtype=np.int64) for _, _, g in live])
    order = np.lexsort((local, rank, seq))   # seq, then rank, then the rank's own order
    cols = [np.concatenate([rows[k] for _, rows, _ in live])[order] for k in range(5)]
    ch, rk = cols[0], rank[order]
    new = np.r_[True, (ch[1:] != ch[:-1]) | (rk[1:] != rk[:-1])] if len(ch) else np.zeros(0, bool)
    cols[0] = np.cumsum(new) - 1
    return tuple(cols) + (seq[order],)


def call_offsets_from_seq(seq: torch.Tensor, call_size: int) -> torch.Tensor:
    """InputHandler-call boundaries of a seq-sorted event slice: calls of the
    global stream are consecutive runs of `call_size` sequence numbers."""
    n = seq.numel()
    if n == 0:
        return torch.zeros(1, dtype=torch.int64)
    call = seq // call_size
    starts = torch.nonzero(torch.cat([torch.ones(1, dtype=torch.bool, device=seq.device),
                                      call[1:] != call[:-1]])).flatten()
    return torch.cat([starts.to(torch.int64).cpu(), torch.tensor([n], dtype=torch.int64)])


# ---------------------------------------------------------------- HIP routing
def _widths(cols):
    w = []
    for c in cols:
        if c.element_size() not in (4, 8) or not c.is_contiguous():
            raise ValueError("route_device: contiguous 4- or 8-byte columns only")
        w.append(c.element_size())
    return w


def bucket(cols: List[torch.Tensor], key: torch.Tensor, seq: torch.Tensor, world: int, seq_lo: int,
           device: int = 0):
    """shd_route_bucket on torch's current stream: (send words [n * words] int64,
    counts [world] int64 device, words per row)."""
    import ctypes
    from siddhi_amd import hip_engine as he
    lib, ctx = he.load_library(), he.context(device)
    n = seq.numel()
    widths = _widths(cols)
    wa = (ctypes.c_int * max(len(cols), 1))(*widths)
    words = ctypes.c_int()
    he._check(lib.shd_route_words(len(cols), wa, ctypes.byref(words)))
    send = torch.empty(max(n, 1) * words.value, dtype=torch.int64, device=seq.device)
    counts = torch.empty(world, dtype=torch.int64, device=seq.device)
    ptrs = (ctypes.c_void_p * max(len(cols), 1))(*[c.data_ptr() for c in cols])
    if key.dtype not in (torch.int32, torch.int64) or not key.is_contiguous() or not seq.is_contiguous():
        raise ValueError("route_device: contiguous int32/int64 key and int64 seq")
    sb = ctypes.c_size_t()
    he._check(lib.shd_route_bucket_scratch(n, world, ctypes.byref(sb)))
    scratch = torch.empty((sb.value + 7) // 8, dtype=torch.int64, device=seq.device)
    stream = torch.cuda.current_stream(seq.device).cuda_stream
    he._check(lib.shd_route_bucket(ctx, stream, n, world, key.data_ptr(), key.element_size(), len(cols), ptrs, wa,
                                   seq.data_ptr(), int(seq_lo), send.data_ptr(), counts.data_ptr(),
                                   scratch.data_ptr()))
    return send[:n * words.value], counts, words.value


class HostCopy:
    """A device -> pinned-host copy enqueued on the current stream, with an
    event behind it: get() waits only for that event, and a pipelined caller
    asks one micro-batch later, when the copy has long landed -- no
    synchronous device-to-host read on the route's critical path."""

    def __init__(self, t: torch.Tensor):
        self.host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        self.host.copy_(t, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()

    def get(self) -> torch.Tensor:
        self.event.synchronize()
        return self.host


class CallOffsets:
    """The merged micro-batch's InputHandler-call offsets, read from the
    merge's tail (block offsets + error flag) once its HostCopy landed;
    `event`: recorded after the merge on the route's stream (a consumer on
    another stream waits on it instead of synchronising the host)."""

    def __init__(self, tail: HostCopy, nblocks: int):
        self._tail, self._nb, self._co = tail, nblocks, None
        self.event = tail.event

    def get(self):
        import numpy as np
        if self._co is None:
            th = self._tail.get().numpy()
            nb = self._nb
            if int(th[nb + 1:].view(np.int32)[0]) != 0:
                raise ValueError("route_device: received rows outside the micro-batch's calls (seq_lo / nblocks)")
            co = np.unique(th[:nb + 1])
            if len(co) == 0 or co[0] != 0:
                co = np.concatenate([[0], co])
            self._co = co.astype(np.int64)
        return self._co


def merge(recv: torch.Tensor, recv_counts: torch.Tensor, dtypes: List[torch.dtype], world: int, seq_lo: int,
          call_size: int, nblocks: int, device: int = 0, m: Optional[int] = None, lazy: bool = False):
    """shd_route_merge on torch's current stream: the received rows of `world`
    senders (sender s's recv_counts[s] rows in turn) in global sequence order.
    m: total rows when the caller knows it (saves a device read).
    Returns (columns, seq, call offsets as a host int64 array; lazy: a
    CallOffsets whose copy is still in flight)."""
    import ctypes
    import numpy as np
    from siddhi_amd import hip_engine as he
    lib, ctx = he.load_library(), he.context(device)
    dev = recv.device
    seg_off = torch.zeros(world + 1, dtype=torch.int64, device=dev)
    seg_off[1:] = torch.cumsum(recv_counts, 0)
    if m is None:
        m = int(seg_off[-1].item())
    outs = [torch.empty(m, dtype=dt, device=dev) for dt in dtypes]
    widths = _widths(outs)
    wa = (ctypes.c_int * max(len(outs), 1))(*widths)
    ptrs = (ctypes.c_void_p * max(len(outs), 1))(*[c.data_ptr() for c in outs])
    out_seq = torch.empty(m, dtype=torch.int64, device=dev)
    start = torch.empty((nblocks + 1) * world, dtype=torch.int64, device=dev)
    # call offsets and the error flag (last word) come back in ONE device -> host copy
    tail = torch.empty(nblocks + 2, dtype=torch.int64, device=dev)
    block_off, err = tail[:nblocks + 1], tail[nblocks + 1:].view(torch.int32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    he._check(lib.shd_route_merge(ctx, stream, world, recv.data_ptr(), seg_off.data_ptr(), m, int(seq_lo),
                                  int(call_size), int(nblocks), len(outs), ptrs, wa, out_seq.data_ptr(),
                                  start.data_ptr(), block_off.data_ptr(), err.data_ptr()))
    co = CallOffsets(HostCopy(tail), nblocks)
    return outs, out_seq, (co if lazy else co.get())


def route_stage_a(cols: List[torch.Tensor], key: torch.Tensor, seq: torch.Tensor, world: int, seq_lo: int,
                  group: Optional[dist.ProcessGroup] = None, device: int = 0, stage_host: bool = False) -> dict:
    """Route, first half: HIP bucket by owner + the all-to-all of the
    per-owner counts; both counts vectors go to pinned host memory without
    waiting (HostCopy) -- stage B of the same micro-batch, issued one
    micro-batch later in a pipeline, sizes the data exchange from them."""
    st = {"dtypes": [c.dtype for c in cols], "n": seq.numel(), "world": world, "seq_lo": seq_lo,
          "group": group, "device": device, "stage_host": stage_host}
    send, counts, words = bucket(cols, key, seq, world, seq_lo, device)
    st.update(send=send, counts=counts, words=words)
    if world > 1:
        recv_counts = torch.empty_like(counts)
        _a2a(recv_counts, counts, group=group, stage_host=stage_host)
        st["recv_counts"] = recv_counts
        st["host_counts"] = HostCopy(torch.cat([counts, recv_counts]))
    return st


def _a2a(out, inp, out_splits=None, in_splits=None, group=None, stage_host=False):
    if not stage_host:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
        return
    ho = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(ho, inp.cpu(), out_splits, in_splits, group=group)
    out.copy_(ho)


def route_stage_b(st: dict, call_size: int, nblocks: int, lazy: bool = True):
    """Route, second half: the data all-to-all (split sizes from stage A's
    host counts), then the HIP merge into global sequence order.  lazy: the
    call offsets come back as a CallOffsets (copy in flight)."""
    world, group, device = st["world"], st["group"], st["device"]
    send, counts, words = st["send"], st["counts"], st["words"]
    if world > 1:
        hc = st["host_counts"].get().tolist()
        cs, rcs = hc[:world], hc[world:]
        recv = torch.empty(sum(rcs) * words, dtype=torch.int64, device=send.device)
        _a2a(recv, send, [c * words for c in rcs], [c * words for c in cs], group=group,
             stage_host=st["stage_host"])
        rank = dist.get_rank(group)
        stats = {"sent": sum(cs) - cs[rank], "received": sum(rcs) - rcs[rank]}
        recv_counts, m = st["recv_counts"], sum(rcs)
    else:
        recv, recv_counts, stats, m = send, counts, {"sent": 0, "received": 0}, st["n"]
    outs, rseq, co = merge(recv, recv_counts, st["dtypes"], world, st["seq_lo"], call_size, nblocks, device, m=m,
                           lazy=lazy)
    return outs, rseq, co, stats


def route_device(cols: List[torch.Tensor], key: torch.Tensor, seq: torch.Tensor, world: int, seq_lo: int,
                 call_size: int, nblocks: int, group: Optional[dist.ProcessGroup] = None, device: int = 0,
                 stage_host: bool = False):
    """route() on the GPU with the HIP bucket / merge passes around ONE RCCL
    all-to-all (plus the all-to-all of the per-owner counts, whose host copy
    sizes the exchange).  The micro-batch's events hold sequence numbers in
    [seq_lo, seq_lo + nblocks * call_size) with seq_lo a multiple of call_size
    (the global stream's InputHandler calls).  Returns (columns, seq, host call
    offsets, stats) in increasing sequence order.  The two stages
    (route_stage_a / route_stage_b) run back to back here; RoutePipeline.run_staged
    interleaves them across micro-batches so nothing waits on the device.
    stage_host: the two all-to-alls run on host copies (a gloo group, e.g. ranks
    sharing one GPU in tests; RCCL needs one GPU per rank)."""
    st = route_stage_a(cols, key, seq, world, seq_lo, group, device, stage_host)
    outs, rseq, co, stats = route_stage_b(st, call_size, nblocks, lazy=False)
    return outs, rseq, co, stats


class RoutePipeline:
    """Micro-batch k+1's route (HIP bucket -> all-to-alls -> HIP merge) runs on a
    side stream in a worker thread while the caller pushes micro-batch k: the
    exchange overlaps the engine push.  The route's host reads -- the per-owner
    counts that size the all-to-all and the merged call offsets -- happen in
    the worker, off the push's critical path; nothing between the caller's
    previous push and its next one waits on a device-to-host copy.  The worker
    issues the collectives in micro-batch order (one thread: the same order on
    every rank).  Usage: ``for routed in pipe.run(jobs): push(routed)`` where a
    job is a no-argument callable returning route_device()'s result.
    Lifetime: the routed tensors live on the side stream's pool; the engine
    reads them on its own stream, so the caller keeps micro-batch k's result
    referenced until its NEXT push has returned (every shd_push synchronises
    the engine's stream at least once, so push k + 1 returning means push k's
    kernels are done): only then may the allocator hand k's memory to the
    route of a later micro-batch (bench.py run_step holds it that way)."""

    def __init__(self, device: int = 0):
        from concurrent.futures import ThreadPoolExecutor
        self.device = device
        self.stream = torch.cuda.Stream(device=device)
        self.pool = ThreadPoolExecutor(max_workers=1)

    def _route(self, job):
        torch.cuda.set_device(self.device)
        with torch.cuda.stream(self.stream):
            r = job()
        self.stream.synchronize()   # routed columns complete before another stream reads them
        return r

    def _staged(self, jobs, i):
        """Worker step i: stage A of micro-batch i + 1, then stage B of i (whose
        host counts were copied during step i - 1).  The routed columns are
        fenced with an event on the side stream, not a host sync."""
        torch.cuda.set_device(self.device)
        with torch.cuda.stream(self.stream):
            if i == 0:
                self._st[0] = jobs[0][0]()
            if i + 1 < len(jobs):
                self._st[i + 1] = jobs[i + 1][0]()
            r = jobs[i][1](self._st.pop(i))
        return r

    def run_staged(self, jobs):
        """jobs: (stage_a, stage_b) pairs -- stage_a() -> state (route_stage_a),
        stage_b(state) -> route result with lazy CallOffsets (route_stage_b).
        The collectives keep micro-batch order on every rank: counts of i + 1
        before the data of i.  The caller makes its engine stream wait on
        result[2].event and reads result[2].get() when it pushes."""
        self._st = {}
        pending = None
        for i in range(len(jobs)):
            nxt = self.pool.submit(self._staged, jobs, i)
            if pending is not None:
                yield pending.result()
            pending = nxt
        if pending is not None:
            yield pending.result()

    def run(self, jobs):
        pending = None
        for job in jobs:
            nxt = self.pool.submit(self._route, job)   # k+1 starts before k is handed out
            if pending is not None:
                yield pending.result()
            pending = nxt
        if pending is not None:
            yield pending.result()

    def close(self):
        self.pool.shutdown(wait=True)


# ---------------------------------------------------------------------------
# Time slices with a halo: unpartitioned window aggregates (configs W2-*).
#
# A window query without a partition holds ONE window over the whole stream
# (LengthWindowProcessor / TimeWindowProcessor state is per query, C/query/
# processor/stream/window/LengthWindowProcessor.java:106-142), so its events
# cannot be split by key.  They split by time instead: rank r takes the
# contiguous slice r of the global stream (cut on InputHandler-call
# boundaries).  Everything the slice's rows depend on besides its own events is
# the window content when the slice starts -- the last L filter-passing events
# (length) or the events of the last T ms (time) -- and all of that lies in the
# tail of slice r-1.  Rank r-1 sends that tail (the halo, one point-to-point
# pair per rank and step: the only data-path exchange), rank r pushes it
# through a fresh query first and drops its rows, then pushes its own slice:
# from there on the query's state equals the one-engine state at that point
# (length: the same L items; time: every item not yet expired), so rank r's
# rows are exactly the one-engine rows of its calls, and the ranks' rows
# concatenated in rank order are the whole stream's.  The halo's size is found
# once (`halo_take`): double it until every rank's halo covers its window.
# ---------------------------------------------------------------------------

def window_of(qp) -> Optional[Tuple[str, int]]:
    """("length", L) or ("time", T ms) of a single-stream window query (planner
    Plan.handlers), None without a window."""
    from . import planner as pl
    for h in qp.plan.handlers:
        if h[0] == pl.H_WINDOW:
            if h[1] not in (pl.W_LENGTH, pl.W_TIME):
                raise pl.UnsupportedPlanException("slices with a halo need a sliding length / time window")
            return ("length" if h[1] == pl.W_LENGTH else "time", int(h[2]))
    return None


def _peer(rank: int, group: Optional[dist.ProcessGroup]) -> int:
    """Global rank of group rank `rank` (P2POp addresses global ranks)."""
    return rank if group is None else dist.get_global_rank(group, rank)


def exchange_tail(cols: List[torch.Tensor], take: int, rank: int, world: int,
                  group: Optional[dist.ProcessGroup] = None,
                  nulls: Optional[List[Optional[torch.Tensor]]] = None):
    """Rank r (its rank in `group`) sends the last `take` rows of its slice to
    rank r+1 and receives rank r-1's (None on rank 0).  `take` must be the
    same on every rank and at most every rank's slice length (halo_take
    returns such a size); columns travel packed (pack()).  nulls: per-column
    null masks (None = no nulls); they travel as one extra bit-mask column
    (as in route()) and the call returns (columns, masks): a halo row whose
    value is null must prime the query as null, not as its placeholder value."""
    if nulls is not None:
        if len(nulls) != len(cols) or len(cols) > 62:
            raise ValueError("one null mask (or None) per column, at most 62 columns")
        bits = torch.zeros(cols[0].numel(), dtype=torch.int64, device=cols[0].device)
        for j, m in enumerate(nulls):
            if m is not None:
                bits |= m.to(torch.int64) << j
        got = exchange_tail(list(cols) + [bits], take, rank, world, group)
        if got is None:
            return None
        rb = got.pop()
        return got, [((rb >> j) & 1).to(torch.uint8) for j in range(len(cols))]
    dtypes = [c.dtype for c in cols]
    if take <= 0 or world == 1:
        return None
    if take > cols[0].numel():
        raise ValueError("halo of %d rows from a slice of %d" % (take, cols[0].numel()))
    ops, recv = [], None
    if rank + 1 < world:
        ops.append(dist.P2POp(dist.isend, pack([c[-take:] for c in cols]), _peer(rank + 1, group), group))
    if rank > 0:
        recv = torch.empty((take, len(cols)), dtype=torch.int64, device=cols[0].device)
        ops.append(dist.P2POp(dist.irecv, recv, _peer(rank - 1, group), group))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return None if recv is None else unpack(recv, dtypes)


def halo_covers(window: Tuple[str, int], carry: int, halo_ts: torch.Tensor, first_ts: int) -> bool:
    """True when a halo leaves the window exactly as one engine has it before the
    slice's first event.  length: the query holds L items after the halo
    (counters.carry, the items its window carries).  time: with nondecreasing
    timestamps, the halo's first event -- and so every event before it -- has
    expired (ts + T - now <= 0, C/query/processor/stream/window/TimeWindowProcessor.java:144-145) before the
    slice's first event arrives; the margin of one ms keeps it strict."""
    kind, w = window
    if kind == "length":
        return carry >= w
    ts = halo_ts
    if ts.numel() == 0:
        return False
    mono = bool((ts[1:] >= ts[:-1]).all().item()) and int(ts[-1].item()) <= first_ts
    return mono and int(ts[0].item()) + w < first_ts


def halo_take(window: Tuple[str, int], n: int, exchange, prime, device=None,
              group: Optional[dist.ProcessGroup] = None, start: int = 0) -> int:
    """The halo size (events) every rank uses: the smallest power-of-two
    multiple of `start` (default 2L for length windows, 4096 events for time)
    at which every rank's halo covers its window.  exchange(take) -> the
    received halo columns (None on rank 0); prime(halo) -> bool, the
    halo_covers() verdict after pushing `halo` into a fresh query.  Raises when
    a whole previous slice is not enough (the window reaches back past it).
    Slices may differ in length (a stream that does not divide evenly): every
    rank works with the shortest slice length, so every rank computes the same
    sizes, sends as many rows as its successor expects and takes the raise
    branch together."""
    if device is None and dist.get_backend(group) != "gloo":
        device = torch.device("cuda", torch.cuda.current_device())   # RCCL reduces device tensors only
    nt = torch.tensor([int(n)], dtype=torch.int64, device=device)
    dist.all_reduce(nt, op=dist.ReduceOp.MIN, group=group)
    n = int(nt.item())
    take = min(n, start or (2 * window[1] if window[0] == "length" else 4096))
    while True:
        halo = exchange(take)
        ok = True if halo is None else bool(prime(halo))
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag.item()) == 0:
            return take
        if take >= n:
            raise ValueError("window reaches back past the previous rank's whole slice (%d events)" % n)
        take = min(n, take * 2)
