"""Host-side mirror of the reference API for the hot path.

SiddhiManager / SiddhiAppRuntime / InputHandler / QueryCallback / StreamCallback
with the reference's names, argument meaning and error behaviour
(C/SiddhiManager.java:84-96, C/SiddhiAppRuntimeImpl.java:260-269,414-415,
C/stream/input/InputHandler.java:50-95, C/query/output/callback/QueryCallback.java:61-106,
C/stream/output/StreamCallback.java:93-129).

Every query is executed by a query engine.  The product engine is
`siddhi_amd.hip_engine.HipQueryEngine` (libsiddhi_hip, MI355X); there is no CPU
fallback: if the HIP library cannot be loaded the runtime raises.  Tests may
pass another engine factory (the CPU oracle) explicitly as a checker.

Junction semantics (C/stream/StreamJunction.java:146-272): synchronous fan-out
to subscribed queries in definition order; query outputs are delivered to the
target stream's junction within the same call.  Time (playback,
C/util/timestamp/TimestampGeneratorImpl.java:58-76): every InputHandler.send
advances the app clock to the last event's timestamp and fires every query's
due timers before the events are routed.
"""
from __future__ import annotations

import hashlib
import json
import struct
import time
from typing import Callable, Dict, List, Optional

import numpy as np

from . import planner as pl
from . import query_compiler as qc

CURRENT, EXPIRED = 0, 1


class Event:
    """io.siddhi.core.event.Event"""

    __slots__ = ("timestamp", "data", "is_expired")

    def __init__(self, timestamp: int = -1, data=None, is_expired: bool = False):
        self.timestamp = int(timestamp)
        self.data = list(data) if data is not None else []
        self.is_expired = is_expired

    def getTimestamp(self):
        return self.timestamp

    def getData(self, i=None):
        return self.data if i is None else self.data[i]

    def isExpired(self):
        return self.is_expired

    def __repr__(self):
        return "Event{timestamp=%d, data=%r, isExpired=%s}" % (self.timestamp, self.data, self.is_expired)


class QueryCallback:
    """io.siddhi.core.query.output.callback.QueryCallback"""

    def receive(self, timestamp, inEvents, removeEvents):  # noqa: N802,N803
        raise NotImplementedError


class StreamCallback:
    """io.siddhi.core.stream.output.StreamCallback"""

    def receive(self, events):
        raise NotImplementedError


class _FnQueryCallback(QueryCallback):
    def __init__(self, fn):
        self.fn = fn

    def receive(self, timestamp, inEvents, removeEvents):
        self.fn(timestamp, inEvents, removeEvents)


class _FnStreamCallback(StreamCallback):
    def __init__(self, fn):
        self.fn = fn

    def receive(self, events):
        self.fn(events)


# ---------------------------------------------------------------- columns
_NP = {pl.T_STRING: np.uint32, pl.T_INT: np.int32, pl.T_LONG: np.int64, pl.T_FLOAT: np.float32,
       pl.T_DOUBLE: np.float64, pl.T_BOOL: np.uint8}


class ColumnBatch:
    """Columnar micro-batch of one stream (SoA), the unit handed to engines."""

    def __init__(self, ts: np.ndarray, cols: List[np.ndarray], nulls: List[Optional[np.ndarray]],
                 call_offsets: Optional[np.ndarray] = None):
        self.ts = ts
        self.cols = cols
        self.nulls = nulls
        self.n = len(ts)
        self.call_offsets = call_offsets if call_offsets is not None else np.array([0, self.n], np.int64)


def _java_value(v, t, dictionary):
    if v is None:
        return None
    if t == pl.T_STRING:
        return dictionary.id(str(v))
    if t == pl.T_BOOL:
        return 1 if v else 0
    if t == pl.T_INT:
        iv = int(v)
        return ((iv + 2 ** 31) % 2 ** 32) - 2 ** 31
    if t == pl.T_LONG:
        return int(v)
    return float(v)


def rows_to_batch(types: List[int], events: List[Event], dictionary) -> ColumnBatch:
    """Event[] of one InputHandler call -> SoA batch (StreamEventConverter's
    job, C/event/stream/converter/SimpleStreamEventConverter.java:36-42)."""
    n = len(events)
    ts = np.fromiter((e.timestamp for e in events), np.int64, n)
    cols, nulls = [], []
    for a, t in enumerate(types):
        raw = [e.data[a] if a < len(e.data) else None for e in events]
        nm = np.fromiter((x is None for x in raw), np.uint8, n)
        has_null = bool(nm.any())
        if t == pl.T_STRING:
            ids = dictionary.ids
            col = np.fromiter((0 if x is None else (ids.get(x) if type(x) is str and x in ids else
                                                    dictionary.id(str(x))) for x in raw), np.uint32, n)
        elif t == pl.T_DOUBLE and not has_null and all(type(x) is float for x in raw):
            col = np.array(raw, np.float64)
        elif t in (pl.T_LONG, pl.T_INT) and not has_null and all(type(x) is int for x in raw):
            try:   # in range: the values as they are (no Java int wrap needed)
                col = np.array(raw, dtype=_NP[t])
            except OverflowError:
                col = np.array([_java_value(x, t, dictionary) for x in raw], dtype=_NP[t])
        else:
            col = np.array([0 if x is None else _java_value(x, t, dictionary) for x in raw], dtype=_NP[t])
        cols.append(col)
        nulls.append(nm if has_null else None)
    return ColumnBatch(ts, cols, nulls)


def decode_value(bits: int, t: int, dictionary):
    bits = int(bits) & ((1 << 64) - 1)
    if t == pl.T_STRING:
        return dictionary.lookup(bits)
    if t == pl.T_INT:
        v = bits & 0xFFFFFFFF
        return v - (1 << 32) if v >= (1 << 31) else v
    if t == pl.T_LONG:
        return bits - (1 << 64) if bits >= (1 << 63) else bits
    if t == pl.T_FLOAT:
        return float(np.array([bits & 0xFFFFFFFF], np.uint32).view(np.float32)[0])
    if t == pl.T_DOUBLE:
        return float(np.array([bits], np.uint64).view(np.float64)[0])
    if t == pl.T_BOOL:
        return bool(bits)
    raise ValueError(t)


class OutputChunk:
    """One callback invocation worth of output rows (ComplexEventChunk)."""

    __slots__ = ("types", "ts", "values", "nulls", "objects")

    def __init__(self, types, ts, values, nulls, objects=None):
        self.types = types      # np.int32 [n] CURRENT / EXPIRED
        self.ts = ts            # np.int64 [n]
        self.values = values    # np.uint64 [n, n_out] bit patterns
        self.nulls = nulls      # np.uint8 [n, n_out]
        # OBJECT columns (multi-value selections): col -> per row a list of
        # (bits, null) element payloads
        self.objects = objects or {}


def list_columns(qp) -> Dict[int, int]:
    """Output columns of type OBJECT (multi-value selections of a count
    state, include/siddhi_ir.h SHD_OP_MULTI) -> their element type."""
    out = {}
    for k, (_, t, e) in enumerate(qp.plan.outputs):
        if t == pl.T_OBJECT:
            out[k] = qp.plan.exprs[e][0][3] >> 16
    return out


def decode_lists(vals, cols, lvals, lnul) -> Dict[int, list]:
    """Per OBJECT column, per row: the list its handle (offset | count << 40)
    addresses in the list arena, as (bits, null) pairs."""
    out = {}
    for k in cols:
        rows = []
        for h in vals[:, k]:
            h = int(h)
            off, cnt = h & ((1 << 40) - 1), h >> 40
            rows.append([(int(lvals[off + j]), bool(lnul[off + j])) for j in range(cnt)])
        out[k] = rows
    return out


def split_chunks(chunk_ids, types, ts, vals, nulls, objects=None) -> List[OutputChunk]:
    out = []
    n = len(chunk_ids)
    if n == 0:
        return out
    starts = np.flatnonzero(np.r_[True, chunk_ids[1:] != chunk_ids[:-1]])
    ends = np.r_[starts[1:], n]
    for s, e in zip(starts, ends):
        obj = {k: v[s:e] for k, v in objects.items()} if objects else None
        out.append(OutputChunk(types[s:e], ts[s:e], vals[s:e], nulls[s:e], obj))
    return out


# ---------------------------------------------------------------- runtime
class _QueryRuntime:
    def __init__(self, qp: pl.QueryPlan, engine, name):
        self.qp = qp
        self.engine = engine
        self.name = name
        self.callbacks: List[QueryCallback] = []
        rate = getattr(qp, "output_rate", None)
        self.limiter = OutputRateLimiter(rate, qp.rate_group_cols is not None) if rate is not None else None
        self.list_cols = list_columns(qp) if pl.T_OBJECT in qp.output_types else {}


class InputHandler:
    """io.siddhi.core.stream.input.InputHandler (C/stream/input/InputHandler.java:50-95)."""

    def __init__(self, runtime: "SiddhiAppRuntime", stream_id: str):
        self._rt = runtime
        self.stream_id = stream_id

    def getStreamId(self):
        return self.stream_id

    def send(self, *args):
        """send(Object[] data) | send(long ts, Object[] data) | send(Event) | send(Event[])."""
        if len(args) == 2:
            evs = [Event(args[0], args[1])]
        elif len(args) == 1:
            a = args[0]
            if isinstance(a, Event):
                evs = [a]
            elif isinstance(a, (list, tuple)) and a and isinstance(a[0], Event):
                evs = list(a)
            elif isinstance(a, (list, tuple)) and not a:
                return
            else:
                evs = [Event(self._rt._wall_clock(), a)]
        else:
            raise TypeError("send(data) | send(ts, data) | send(Event) | send(Event[])")
        self._rt._send(self.stream_id, evs)

    def send_batch(self, batch: ColumnBatch):
        """Columnar fast path: one pre-built SoA batch (call boundaries in batch.call_offsets)."""
        if not self._rt.started:
            raise RuntimeError("Siddhi app '%s' is not running, cannot send events" % self._rt.name)
        self._rt._send_columns(self.stream_id, batch)


def _duration_ms(text: str) -> int:
    """'100 millisecond' / '2 sec' / '500' (ms) -> milliseconds."""
    parts = str(text).strip().split()
    n = int(float(parts[0]))
    if len(parts) == 1:
        return n
    unit = qc._time_unit(parts[1])
    if unit is None:
        raise ValueError("unknown time unit in %r" % text)
    return n * unit


class SiddhiAppRuntime:
    """io.siddhi.core.SiddhiAppRuntime"""

    def __init__(self, app: qc.SiddhiApp, engine_factory: Callable, app_text: str):
        self.app = app
        self.app_text = app_text
        self.dictionary = pl.StringDictionary()
        self.name = None
        ann = app.annotation("app:name")
        if ann is not None and ann.elements:
            self.name = ann.elements[0][1]
        self.playback = app.annotation("app:playback") is not None
        # @app:playback(idle.time = '100 millisecond', increment = '2 sec'): the
        # heartbeat that moves playback time while no events arrive
        # (TimestampGeneratorImpl.setIdleTime / setIncrementInMilliseconds)
        self.idle_time = self.idle_increment = None
        if self.playback:
            pa = app.annotation("app:playback")
            it, inc = pa.get("idle.time"), pa.get("increment")
            if it is not None and inc is not None:
                self.idle_time, self.idle_increment = _duration_ms(it), _duration_ms(inc)
        self._event_time = None   # TimestampGeneratorImpl.lastEventTimestamp (playback)
        self.stream_types: Dict[str, List[int]] = {
            s: [pl.TYPE_CODE[t] for _, t in sd.attrs] for s, sd in app.streams.items()}
        self.queries: List[_QueryRuntime] = []
        self.stream_callbacks: Dict[str, List[StreamCallback]] = {}
        self.subscribers: Dict[str, List[tuple]] = {}
        self.started = False
        self.persistence_store = None
        self._last_wall = 0
        self.clock = None   # wall-clock source (ms); None = time.time() (tests replay a recorded clock)
        extra = {}
        anon = 0
        for item in app.execution_order:
            part = item if isinstance(item, qc.Partition) else None
            qs = item.queries if part else [item]
            for q in qs:
                # output stream definitions are inferred (QueryParser: OutputStream definition)
                qp = pl.plan_query(app, q, self.dictionary, part, extra)
                if q.target not in app.streams and q.target not in extra:
                    extra[q.target] = qc.StreamDef(q.target, [(n, pl.TYPE_NAME[t]) for n, t in
                                                              zip(qp.output_names, qp.output_types)])
                    self.stream_types[q.target] = list(qp.output_types)
                name = q.name or "query_%d" % anon
                anon += 1
                engine = engine_factory(qp, self.dictionary)
                qr = _QueryRuntime(qp, engine, name)
                self.queries.append(qr)
                for si, sid in enumerate(qp.input_streams):
                    self.subscribers.setdefault(sid, []).append((qr, si))

    # -- public API
    def getName(self):
        return self.name

    def addCallback(self, name: str, callback):
        if callable(callback) and not isinstance(callback, (QueryCallback, StreamCallback)):
            raise TypeError("callback must be a QueryCallback or StreamCallback")
        if isinstance(callback, QueryCallback):
            for q in self.queries:
                if q.name == name:
                    q.callbacks.append(callback)
                    return
            raise pl.SiddhiAppCreationException("No query with name '%s' exists" % name)
        if isinstance(callback, StreamCallback):
            if name not in self.stream_types:
                raise pl.SiddhiAppCreationException("Stream with stream ID '%s' has not been defined" % name)
            self.stream_callbacks.setdefault(name, []).append(callback)
            return
        raise TypeError("unknown callback type")

    def getInputHandler(self, stream_id: str) -> InputHandler:
        if stream_id not in self.stream_types:
            raise pl.SiddhiAppCreationException("Stream with stream ID %s has not been defined" % stream_id)
        return InputHandler(self, stream_id)

    def start(self):
        """SiddhiAppRuntime.start(): queries start at the app's current time --
        0 for playback apps (TimestampGeneratorImpl.lastEventTimestamp before
        any event), the wall clock otherwise (C/util/timestamp/TimestampGeneratorImpl.java)."""
        t0 = 0 if self.playback else self._wall_clock()
        for q in self.queries:
            st = getattr(q.engine, "start", None)
            if st:
                st(t0)
            if q.limiter is not None:
                q.limiter.start(self._wall_clock())
        self.started = True

    # -- state persistence (C/SiddhiAppRuntimeImpl.java:677-745)
    _SNAP_MAGIC = b"SIDDHI-AMD-SNAPSHOT-1\n"

    def snapshot(self) -> bytes:
        """SiddhiAppRuntime.snapshot(): the full state of every query (device
        partial-match tables, window contents, aggregates, arrival/time
        counters) plus the host string dictionary the device ids refer to."""
        blobs = [q.engine.snapshot() for q in self.queries]
        head = {"app": hashlib.sha256(self.app_text.encode()).hexdigest(),
                "dictionary": self.dictionary.strings, "last_wall": self._last_wall,
                "queries": [q.name for q in self.queries], "sizes": [len(b) for b in blobs],
                # host-side output rate limiters (their RateLimiterState maps)
                "limiters": {q.name: q.limiter.state() for q in self.queries if q.limiter is not None}}
        hb = json.dumps(head).encode()
        return self._SNAP_MAGIC + struct.pack("<Q", len(hb)) + hb + b"".join(blobs)

    def restore(self, snapshot: bytes):
        """SiddhiAppRuntime.restore(byte[]) (SnapshotService.restore, C/util/snapshot/SnapshotService.java:333)."""
        m = self._SNAP_MAGIC
        if not snapshot.startswith(m):
            raise CannotRestoreSiddhiAppStateException("not a siddhi_amd snapshot")
        (hl,) = struct.unpack_from("<Q", snapshot, len(m))
        at = len(m) + 8
        head = json.loads(snapshot[at:at + hl].decode())
        at += hl
        if head["app"] != hashlib.sha256(self.app_text.encode()).hexdigest() or \
                head["queries"] != [q.name for q in self.queries]:
            raise CannotRestoreSiddhiAppStateException("snapshot was taken from a different Siddhi app")
        strings = head["dictionary"]
        cur = self.dictionary.strings
        # the device state holds dictionary ids: they keep their meaning when
        # either dictionary is a prefix of the other (strings interned after
        # persist(), or before a restore into a fresh runtime, only append)
        k = min(len(strings), len(cur))
        if strings[:k] != cur[:k]:
            raise CannotRestoreSiddhiAppStateException("string dictionary of the snapshot conflicts with this app's")
        sizes = head["sizes"]
        if len(sizes) != len(self.queries) or at + sum(sizes) != len(snapshot):
            raise CannotRestoreSiddhiAppStateException("snapshot is truncated or has trailing bytes")
        for x in strings[len(cur):]:
            self.dictionary.id(x)
        self._last_wall = max(self._last_wall, int(head["last_wall"]))
        for q, n in zip(self.queries, sizes):
            q.engine.restore(snapshot[at:at + n])
            at += n
        lim = head.get("limiters", {})
        for q in self.queries:
            if q.limiter is not None and q.name in lim:
                q.limiter.load(lim[q.name])

    def persist(self) -> "PersistenceReference":
        """SiddhiAppRuntime.persist(): snapshot saved to the manager's persistence store."""
        store = self._store()
        rev = "%d_%s" % (int(time.time() * 1000), self.name)
        store.save(self.name, rev, self.snapshot())
        return PersistenceReference(rev)

    def restoreRevision(self, revision: str):  # noqa: N802
        data = self._store().load(self.name, revision)
        if data is None:
            raise CannotRestoreSiddhiAppStateException("no revision '%s' for app '%s'" % (revision, self.name))
        self.restore(data)

    def restoreLastRevision(self):  # noqa: N802
        store = self._store()
        rev = store.getLastRevision(self.name)
        if rev is not None:
            self.restore(store.load(self.name, rev))
        return rev

    def clearAllRevisions(self):  # noqa: N802
        self._store().clearAllRevisions(self.name)

    def _store(self):
        if self.persistence_store is None:
            raise NoPersistenceStoreException("No persistence store assigned for siddhi app " + str(self.name))
        return self.persistence_store

    def shutdown(self):
        for q in self.queries:
            close = getattr(q.engine, "close", None)
            if close:
                close()
        self.queries = []
        self.started = False

    def advanceTime(self, ts: int):  # noqa: N802
        """Move the app clock to `ts` and fire every query's due timers (absent
        `not ... for` states, time windows): what the reference's Scheduler does
        when wall-clock time passes (C/util/Scheduler.java:113-209) or a playback
        heartbeat advances TimestampGeneratorImpl (C/util/timestamp/
        TimestampGeneratorImpl.java:58-76)."""
        if not self.started:
            raise RuntimeError("Siddhi app '%s' is not running" % self.name)
        t = int(ts)
        self._last_wall = max(self._last_wall, t)
        if self._event_time is None or t > self._event_time:
            self._event_time = t
        for q in self.queries:
            self._deliver(q, q.engine.set_time(t))
            self._limit_time(q, t)

    def idle(self, ms: int):
        """`ms` of wall-clock time pass with no events on a playback app: its
        heartbeat moves the app time by `increment` once per `idle.time`
        (TimestampGeneratorImpl.TimeInjector.run, C/util/timestamp/
        TimestampGeneratorImpl.java:168-184: each injection re-arms the
        heartbeat for another idle period).  No-op without idle.time."""
        if not self.playback or self.idle_time is None or self._event_time is None:
            return
        for _ in range(int(ms) // max(self.idle_time, 1)):
            self.advanceTime(self._event_time + self.idle_increment)

    # -- internals
    def _wall_clock(self):
        t = int(self.clock()) if self.clock else int(time.time() * 1000)
        self._last_wall = max(self._last_wall, t)
        return self._last_wall

    def _send(self, stream_id, events: List[Event]):
        if not self.started:
            raise RuntimeError("Siddhi app '%s' is not running, cannot send events" % self.name)
        batch = rows_to_batch(self.stream_types[stream_id], events, self.dictionary)
        self._send_columns(stream_id, batch)

    def _send_columns(self, stream_id, batch: ColumnBatch):
        if batch.n == 0:
            return
        offs = batch.call_offsets
        if len(offs) > 2 and self._batch_push_ok(stream_id):
            # several InputHandler calls, one push per query: each engine
            # advances playback time per call itself (shd_batch.call_offsets +
            # advance_time: setCurrentTimestamp before each call's events,
            # InputHandler.java:85-95); with no query chained to another and
            # no rate limiter, every query's chunks are the per-call path's
            ends = np.asarray(offs[1:], np.int64) - 1
            t = int(np.max(batch.ts[ends]))
            if self._event_time is None or t > self._event_time:
                self._event_time = t
            subs = {id(q): si for q, si in self.subscribers.get(stream_id, [])}
            for q in self.queries:
                if q.limiter is not None:
                    continue
                si = subs.get(id(q))
                if si is None:
                    # not fed by this stream: its clock still moves call by call
                    # (a TIMER's expired rows carry the time it fired at)
                    for tc in batch.ts[ends].tolist():
                        self._deliver(q, q.engine.set_time(tc))
                else:
                    self._deliver(q, q.engine.push(si, batch, advance_time=True))
            return
        if len(offs) > 2:
            # several InputHandler calls in one batch: time advances per call
            for c in range(len(offs) - 1):
                s, e = int(offs[c]), int(offs[c + 1])
                sub = ColumnBatch(batch.ts[s:e], [x[s:e] for x in batch.cols],
                                  [None if x is None else x[s:e] for x in batch.nulls])
                self._send_columns(stream_id, sub)
            return
        # setCurrentTimestamp(last ts): every query's due timers first
        t = int(batch.ts[-1])
        if self._event_time is None or t > self._event_time:
            self._event_time = t
        for q in self.queries:
            self._deliver(q, q.engine.set_time(t))
            self._limit_time(q, t)
        self._junction(stream_id, batch)

    def _batch_push_ok(self, stream_id) -> bool:
        """A multi-call batch may go to each engine as one push: no stream
        callback on the stream (it receives one Event[] per call), no rate
        limiter, no query feeding another query or a stream callback, and
        every engine takes call boundaries itself (HipQueryEngine)."""
        if self.stream_callbacks.get(stream_id):
            return False
        subs = [id(q) for q, _ in self.subscribers.get(stream_id, [])]
        if len(subs) != len(set(subs)):
            return False
        for q in self.queries:
            if q.limiter is not None or not getattr(q.engine, "batch_calls", False):
                return False
            tg = q.qp.target
            if self.stream_callbacks.get(tg) or self.subscribers.get(tg):
                return False
        return True

    def _junction(self, stream_id, batch: ColumnBatch):
        cbs = self.stream_callbacks.get(stream_id)
        if cbs:
            evs = self._batch_events(stream_id, batch)
            for cb in cbs:
                cb.receive(evs)
        for q, si in self.subscribers.get(stream_id, []):
            self._deliver(q, q.engine.push(si, batch))

    def _batch_events(self, stream_id, batch):
        """A batch as the Event[] a StreamCallback receives (column-wise decode)."""
        types = self.stream_types[stream_id]
        cols = []
        for a, t in enumerate(types):
            c = batch.cols[a]
            if t == pl.T_STRING:
                strings = self.dictionary.strings
                vals = [strings[i] for i in c.tolist()]
            elif t == pl.T_BOOL:
                vals = [bool(v) for v in c.tolist()]
            else:
                vals = list(c) if t == pl.T_OBJECT else c.tolist()
            nm = batch.nulls[a]
            if nm is not None and nm.any():
                for i in np.flatnonzero(nm).tolist():
                    vals[i] = None
            cols.append(vals)
        return [Event(t, list(d)) for t, d in zip(batch.ts.tolist(), zip(*cols))]

    def _list_value(self, elems, et):
        """A multi-value cell: the List MultiValueVariableFunctionExecutor returns."""
        return [None if z else decode_value(b, et, self.dictionary) for b, z in elems]

    def _limiter_now(self):
        # TimestampGenerator.currentTime(): event time in playback, else the wall clock
        if self.playback and self._event_time is not None:
            return self._event_time
        return self._wall_clock()

    def _limit_time(self, q: _QueryRuntime, t: int):
        if q.limiter is not None and q.limiter.timed():
            for out in q.limiter.on_time(t):
                self._emit(q, [r[0] for r in out], None, q.list_cols)

    def _deliver(self, q: _QueryRuntime, chunks: List[OutputChunk]):
        if not chunks:
            return
        types = q.qp.output_types
        lcols = q.list_cols
        target = q.qp.target
        chained = target in self.stream_types and bool(self.stream_callbacks.get(target) or
                                                       self.subscribers.get(target))
        for ch in chunks:
            if q.limiter is None and not q.callbacks:
                if chained:
                    self._emit(q, None, ch, lcols)
                continue
            # whole columns decoded at once (QueryCallback.receiveStreamEvent's Event[])
            cols = decode_columns(ch.values, ch.nulls, types, self.dictionary, ch.objects,
                                  lambda elems, k: self._list_value(elems, lcols[k]))
            exp = (ch.types == EXPIRED).tolist()
            evs = [Event(t, list(d), x) for t, d, x in zip(ch.ts.tolist(), zip(*cols), exp)] if cols else \
                [Event(t, [], x) for t, x in zip(ch.ts.tolist(), exp)]
            if q.limiter is None:
                self._emit(q, evs, ch, lcols)
                continue
            gc = q.qp.rate_group_cols
            rows = [(e, tuple(repr(e.data[c]) for c in gc) if gc is not None else None) for e in evs]
            out = q.limiter.process(rows, self._limiter_now())
            if out:
                self._emit(q, [r[0] for r in out], None, lcols)

    def _emit(self, q: _QueryRuntime, evs, ch, lcols):
        """One output chunk to the query's callbacks and its target stream
        (OutputRateLimiter.sendToCallBacks); ch: the engine chunk the events
        are, unchanged (None: rows picked by a rate limiter; evs None: no
        query callback, the chunk only feeds the target stream)."""
        types = q.qp.output_types
        # QueryCallback.receiveStreamEvent (QueryCallback.java:61-91)
        if q.callbacks and evs:
            cur = [e for e in evs if not e.is_expired] or None
            rem = [e for e in evs if e.is_expired] or None
            ts = evs[-1].timestamp
            for cb in q.callbacks:
                cb.receive(ts, cur, rem)
        # InsertIntoStreamCallback: EXPIRED -> CURRENT, into the target junction
        target = q.qp.target
        if not (target in self.stream_types and (self.stream_callbacks.get(target) or self.subscribers.get(target))):
            return
        if ch is None:
            self._junction(target, rows_to_batch(types, [Event(e.timestamp, e.data) for e in evs], self.dictionary))
            return
        cols, nulls = [], []
        for k, t in enumerate(types):
            if t == pl.T_OBJECT:   # java.util.List values travel as objects
                col = np.empty(len(ch.ts), object)
                col[:] = [self._list_value(ch.objects[k][i], lcols[k]) for i in range(len(ch.ts))]
                cols.append(col)
                nulls.append(None)
                continue
            cols.append(_bits_to_col(np.ascontiguousarray(ch.values[:, k], np.uint64), t))
            nm = ch.nulls[:, k].astype(np.uint8)
            nulls.append(nm if nm.any() else None)
        self._junction(target, ColumnBatch(np.asarray(ch.ts, np.int64), cols, nulls))


def _bits_to_col(bits: np.ndarray, t: int) -> np.ndarray:
    if t == pl.T_INT:
        return (bits & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    if t == pl.T_LONG:
        return bits.view(np.int64)
    if t == pl.T_FLOAT:
        return (bits & 0xFFFFFFFF).astype(np.uint32).view(np.float32)
    if t == pl.T_DOUBLE:
        return bits.view(np.float64)
    if t == pl.T_BOOL:
        return bits.astype(np.uint8)
    return bits.astype(np.uint32)


def decode_columns(values: np.ndarray, nulls: np.ndarray, types: List[int], dictionary, objects=None,
                   list_value=None) -> List[list]:
    """Output bit patterns -> the Java values of whole columns (None for
    nulls): decode_value applied per column with NumPy views instead of per
    cell.  OBJECT columns (multi-value lists) go through list_value."""
    n = values.shape[0]
    out = []
    for k, t in enumerate(types):
        if t == pl.T_OBJECT:
            out.append([list_value(objects[k][i], k) for i in range(n)])
            continue
        bits = values[:, k]
        nm = nulls[:, k]
        if t == pl.T_STRING:
            strings = dictionary.strings
            vals = [None if z else strings[i] for i, z in zip(bits.tolist(), nm.tolist())]
        else:
            vals = (bits != 0).tolist() if t == pl.T_BOOL else _bits_to_col(bits, t).tolist()
            if nm.any():
                for i in np.flatnonzero(nm).tolist():
                    vals[i] = None
        out.append(vals)
    return out


class CannotRestoreSiddhiAppStateException(Exception):
    pass


class NoPersistenceStoreException(Exception):
    pass


class PersistenceReference:
    """io.siddhi.core.util.snapshot.PersistenceReference"""

    def __init__(self, revision):
        self.revision = revision

    def getRevision(self):  # noqa: N802
        return self.revision


class InMemoryPersistenceStore:
    """io.siddhi.core.util.persistence.InMemoryPersistenceStore: revisions per app, in order."""

    def __init__(self):
        self._revs: Dict[str, Dict[str, bytes]] = {}

    def save(self, app_name, revision, snapshot: bytes):
        self._revs.setdefault(app_name, {})[revision] = bytes(snapshot)

    def load(self, app_name, revision):
        return self._revs.get(app_name, {}).get(revision)

    def getLastRevision(self, app_name):  # noqa: N802
        revs = self._revs.get(app_name)
        return next(reversed(revs)) if revs else None

    def clearAllRevisions(self, app_name):  # noqa: N802
        self._revs.pop(app_name, None)


class SiddhiManager:
    """io.siddhi.core.SiddhiManager (C/SiddhiManager.java:84-96)."""

    def __init__(self, engine_factory: Optional[Callable] = None, exact_aggregates: bool = False):
        """exact_aggregates: window sum/avg run as the bit-exact sequential
        per-group fold (the reference's add/remove order) instead of the
        default segmented scans (within 1e-9 relative of it)."""
        self._engine_factory = engine_factory
        self._exact_aggregates = exact_aggregates
        self._runtimes: List[SiddhiAppRuntime] = []
        self._store = None

    def setPersistenceStore(self, store):  # noqa: N802
        """SiddhiManager.setPersistenceStore (C/SiddhiManager.java)."""
        self._store = store
        for r in self._runtimes:
            r.persistence_store = store

    def createSiddhiAppRuntime(self, app_text: str) -> SiddhiAppRuntime:
        app = qc.parse(app_text)
        factory = self._engine_factory
        if factory is None:
            from .hip_engine import HipQueryEngine   # product path: MI355X only
            exact = self._exact_aggregates

            def factory(qp, dictionary):
                return HipQueryEngine(qp, dictionary, exact_aggregates=exact)
        rt = SiddhiAppRuntime(app, factory, app_text)
        rt.persistence_store = self._store
        self._runtimes.append(rt)
        return rt

    def shutdown(self):
        for r in self._runtimes:
            r.shutdown()
        self._runtimes = []


# ---------------------------------------------------------------- output rate limiting
class OutputRateLimiter:
    """`output [all|first|last] every <n> events | <time>` on the selector's
    output chunks (C/query/output/ratelimit/{event,time}/*.java), on the host:
    it reorders and drops whole rows the engines already projected.  process()
    takes one selector chunk (rows = (Event, key), key = the group-by values
    for the per-group kinds) and returns the rows to send, as ONE chunk
    (OutputRateLimiter.sendToCallBacks); on_timer() is the Scheduler's TIMER
    (C/util/Scheduler.java:190-220) for the time-based kinds that flush."""

    def __init__(self, rate, grouped: bool):
        self.unit, self.kind, self.value = rate.unit, rate.kind, int(rate.value)
        self.grouped = grouped
        self.counter = 0
        self.buf = []                    # all: the held rows
        self.last = None                 # last (ungrouped, time)
        self.groups = {}                 # first: group -> count / output time; last: group -> row (insertion order)
        self.out_time = None             # first per time (ungrouped)
        self.scheduled = None
        self.notify = []                 # the Scheduler's toNotifyQueue (FIFO)

    def timed(self):
        return self.unit == "time" and self.kind in ("all", "last", "snapshot")

    # -- snapshot / restore: the limiters' RateLimiterState maps
    # (e.g. AllPerTimeOutputRateLimiter.RateLimiterState: the held chunk and
    # scheduledTime; the per-event kinds: counter; the group-by kinds: the
    # per-group maps), as JSON-able values in the runtime's snapshot head
    @staticmethod
    def _row_out(r):
        e, key = r
        return [e.timestamp, e.data, e.is_expired, list(key) if key is not None else None]

    @staticmethod
    def _row_in(x):
        return (Event(x[0], x[1], x[2]), tuple(x[3]) if x[3] is not None else None)

    def _group_vals(self):
        # first: count (per event) / output time (per time); last: the row
        return "row" if self.kind in ("last", "snapshot") else "int"

    def state(self) -> dict:
        gv = self._group_vals()
        return {"counter": self.counter, "buf": [self._row_out(r) for r in self.buf],
                "last": self._row_out(self.last) if self.last is not None else None,
                "groups": [[list(k) if isinstance(k, tuple) else k, self._row_out(v) if gv == "row" else v]
                           for k, v in self.groups.items()],
                "out_time": self.out_time, "scheduled": self.scheduled, "notify": list(self.notify)}

    def load(self, st: dict):
        gv = self._group_vals()
        self.counter = int(st["counter"])
        self.buf = [self._row_in(x) for x in st["buf"]]
        self.last = self._row_in(st["last"]) if st["last"] is not None else None
        self.groups = {(tuple(k) if isinstance(k, list) else k): (self._row_in(v) if gv == "row" else v)
                       for k, v in st["groups"]}
        self.out_time = st["out_time"]
        self.scheduled = st["scheduled"]
        self.notify = list(st["notify"])

    def start(self, wall_now: int):
        # partitionCreated (e.g. AllPerTimeOutputRateLimiter.java:97-108):
        # scheduledTime = System.currentTimeMillis() + value
        if self.timed():
            self.scheduled = wall_now + self.value
            self.notify.append(self.scheduled)

    def process(self, rows, now: int):
        out = []
        if self.unit == "events":
            if self.kind == "all":                       # AllPerEventOutputRateLimiter.process
                for r in rows:
                    self.buf.append(r)
                    self.counter += 1
                    if self.counter == self.value:
                        out += self.buf
                        self.buf, self.counter = [], 0
            elif self.kind == "first" and not self.grouped:   # FirstPerEventOutputRateLimiter
                for r in rows:
                    self.counter += 1
                    if self.counter == 1:
                        out.append(r)
                    elif self.counter == self.value:
                        self.counter = 0
            elif self.kind == "first":                   # FirstGroupByPerEventOutputRateLimiter
                for r in rows:
                    c = self.groups.get(r[1])
                    if c is None:
                        self.groups[r[1]] = 1
                        out.append(r)
                    elif c == self.value - 1:
                        del self.groups[r[1]]
                    else:
                        self.groups[r[1]] = c + 1
            elif not self.grouped:                       # LastPerEventOutputRateLimiter
                for r in rows:
                    self.counter += 1
                    if self.counter == self.value:
                        out.append(r)
                        self.counter = 0
            else:                                        # LastGroupByPerEventOutputRateLimiter
                for r in rows:
                    self.groups[r[1]] = r   # LinkedHashMap.put: a known group keeps its place
                    self.counter += 1
                    if self.counter == self.value:
                        self.counter = 0
                        out += list(self.groups.values())
                        self.groups = {}
            return out
        if self.kind == "snapshot":
            return self._snapshot_rows(rows)
        if self.kind == "all":                           # AllPerTimeOutputRateLimiter
            self.buf += rows
        elif self.kind == "last" and not self.grouped:   # LastPerTimeOutputRateLimiter
            if rows:
                self.last = rows[-1]
        elif self.kind == "last":                        # LastGroupByPerTimeOutputRateLimiter
            for r in rows:
                self.groups[r[1]] = r
        elif not self.grouped:                           # FirstPerTimeOutputRateLimiter: the chunk's first row
            if rows and (self.out_time is None or self.out_time + self.value <= now):
                self.out_time = now
                out.append(rows[0])
        else:                                            # FirstGroupByPerTimeOutputRateLimiter
            for r in rows:
                t0 = self.groups.get(r[1])
                if t0 is None or t0 + self.value <= now:
                    self.groups[r[1]] = now
                    out.append(r)
        return out

    # `output snapshot every <time>` on a non-windowed, non-aggregating query
    # (the planner refuses the rest): PerSnapshotOutputRateLimiter /
    # GroupByPerSnapshotOutputRateLimiter (C/query/output/ratelimit/snapshot/
    # PerSnapshotOutputRateLimiter.java:62-100, GroupByPerSnapshotOutputRateLimiter
    # .java:66-103).  Every event (and TIMER) at or past scheduledTime first
    # flushes a copy of what is held -- the last event, or each group's last
    # event in first-arrival order -- and moves scheduledTime on by one period;
    # a CURRENT event is then held.  The snapshot does not consume what it sends.
    def _snapshot_flush(self):
        out = list(self.groups.values()) if self.grouped else ([self.last] if self.last is not None else [])
        self.scheduled += self.value
        self.notify.append(self.scheduled)
        return out

    def _snapshot_rows(self, rows):
        out = []   # the flushes of one selector chunk go out as one chunk (SnapshotOutputRateLimiter.sendToCallBacks)
        for r in rows:
            if r[0].is_expired:
                # PerSnapshot tries a flush on any other event type; the
                # group-by limiter ignores them
                if not self.grouped and r[0].timestamp >= self.scheduled:
                    out += self._snapshot_flush()
                continue
            if r[0].timestamp >= self.scheduled:
                out += self._snapshot_flush()
            if self.grouped:
                self.groups[r[1]] = r   # LinkedHashMap.put: a known group keeps its place
            else:
                self.last = r
        return out

    def on_time(self, t: int):
        """Due TIMERs up to clock t: the flushed chunks, in order."""
        chunks = []
        while self.notify and self.notify[0] <= t:
            ts = self.notify.pop(0)
            if ts < self.scheduled:
                continue
            if self.kind == "snapshot":   # tryFlushEvents on the TIMER: a copy, nothing consumed
                chunks += [c for c in [self._snapshot_flush()] if c]
                continue
            if self.kind == "all":
                out, self.buf = self.buf, []
            elif not self.grouped:
                out = [self.last] if self.last is not None else []
                self.last = None
            else:
                out, self.groups = list(self.groups.values()), {}
            self.scheduled += self.value
            self.notify.append(self.scheduled)
            if out:
                chunks.append(out)
        return chunks
