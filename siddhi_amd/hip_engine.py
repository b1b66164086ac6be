"""ctypes binding of libsiddhi_hip (include/siddhi_hip.h) and the product
query engine used by SiddhiAppRuntime.

There is no fallback: if the library or a HIP device is missing, loading a
query raises `SiddhiHipError`.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import List

import numpy as np

from . import planner as pl
from .runtime import OutputChunk, decode_lists, list_columns, split_chunks

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHD_LIB") or os.path.join(_HERE, "libsiddhi_hip.so")

SHD_OK, SHD_E_INVALID_PLAN, SHD_E_UNSUPPORTED, SHD_E_OOM, SHD_E_DEVICE, SHD_E_CAPACITY, SHD_E_ARG = \
    0, -1, -2, -3, -4, -5, -6
SHD_MEM_HOST, SHD_MEM_DEVICE = 0, 1
ENGINE_NAMES = {1: "pattern-forward-scan", 2: "window-aggregate", 3: "filter-projection", 4: "nfa"}

EXPORTED = ["shd_device_count", "shd_ctx_create", "shd_ctx_destroy", "shd_plan_load", "shd_plan_free",
            "shd_plan_engine", "shd_set_time", "shd_push", "shd_flush", "shd_poll", "shd_discard_output",
            "shd_reset", "shd_get_counters", "shd_query_stream", "shd_stage_times", "shd_snapshot", "shd_restore",
            "shd_set_option", "shd_route_words", "shd_route_bucket_scratch", "shd_route_bucket", "shd_route_merge",
            "shd_group_create", "shd_group_push", "shd_group_reset", "shd_group_leader", "shd_group_free",
            "shd_last_error"]


class SiddhiHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libsiddhi_hip error %d: %s" % (code, msg))
        self.code = code


class ShdBatch(ctypes.Structure):
    _fields_ = [("stream", ctypes.c_int32), ("mem", ctypes.c_int32), ("n", ctypes.c_int64),
                ("ts", ctypes.c_void_p), ("ncols", ctypes.c_int32), ("cols", ctypes.c_void_p),
                ("nulls", ctypes.c_void_p), ("ncalls", ctypes.c_int32), ("call_offsets", ctypes.c_void_p),
                ("advance_time", ctypes.c_int32), ("use_base_seq", ctypes.c_int32), ("base_seq", ctypes.c_int64)]


class ShdOut(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("n_cols", ctypes.c_int32), ("chunk", ctypes.c_void_p),
                ("type", ctypes.c_void_p), ("ts", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("nulls", ctypes.c_void_p), ("in_seq", ctypes.c_void_p), ("state_idx", ctypes.c_void_p),
                ("n_list", ctypes.c_int64), ("list_values", ctypes.c_void_p), ("list_nulls", ctypes.c_void_p)]


class ShdCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("events", "matches", "partials", "partial_scans", "bytes_touched",
                                               "kernel_ns", "carry", "group_bits", "kernel_ns_total")]


_lib = None
_lib_lock = threading.Lock()
_ctx = None


def load_library(path: str = LIB_PATH):
    """Load libsiddhi_hip.so (raises if missing: the product path has no CPU fallback)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise SiddhiHipError(SHD_E_DEVICE, "%s not built (run __graft_entry__.build())" % path)
        lib = ctypes.CDLL(path)
        P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        lib.shd_device_count.argtypes = [ctypes.POINTER(I)]
        lib.shd_ctx_create.argtypes = [P, I, ctypes.POINTER(P)]
        lib.shd_ctx_destroy.argtypes = [P]
        lib.shd_plan_load.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(P)]
        lib.shd_plan_free.argtypes = [P]
        lib.shd_plan_engine.argtypes = [P, ctypes.POINTER(I)]
        lib.shd_set_time.argtypes = [P, I64]
        lib.shd_set_option.argtypes = [P, ctypes.c_char_p, I64]
        lib.shd_push.argtypes = [P, ctypes.POINTER(ShdBatch)]
        lib.shd_flush.argtypes = [P]
        lib.shd_poll.argtypes = [P, ctypes.POINTER(ShdOut)]
        lib.shd_discard_output.argtypes = [P]
        lib.shd_reset.argtypes = [P]
        lib.shd_get_counters.argtypes = [P, ctypes.POINTER(ShdCounters)]
        lib.shd_query_stream.argtypes = [P, ctypes.POINTER(P)]
        lib.shd_stage_times.argtypes = [P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_char_p), I,
                                        ctypes.POINTER(I)]
        lib.shd_snapshot.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
        lib.shd_restore.argtypes = [P, P, ctypes.c_size_t]
        lib.shd_route_words.argtypes = [I, P, ctypes.POINTER(I)]
        lib.shd_route_bucket_scratch.argtypes = [I64, I, ctypes.POINTER(ctypes.c_size_t)]
        lib.shd_route_bucket.argtypes = [P, P, I64, I, P, I, I, P, P, P, I64, P, P, P]
        lib.shd_route_merge.argtypes = [P, P, I, P, P, I64, I64, I64, I64, I, P, P, P, P, P, P]
        lib.shd_group_create.argtypes = [P, P, ctypes.c_size_t, P, I, ctypes.POINTER(P)]
        lib.shd_group_push.argtypes = [P, ctypes.POINTER(ShdBatch)]
        lib.shd_group_reset.argtypes = [P]
        lib.shd_group_leader.argtypes = [P, ctypes.POINTER(P)]
        lib.shd_group_free.argtypes = [P]
        lib.shd_last_error.restype = ctypes.c_char_p
        for f in EXPORTED:
            if f != "shd_last_error":
                getattr(lib, f).restype = I
        _lib = lib
        return lib


def _check(rc):
    if rc != SHD_OK:
        raise SiddhiHipError(rc, _lib.shd_last_error().decode())


def context(device: int = 0):
    global _ctx
    lib = load_library()
    if _ctx is None:
        ctx = ctypes.c_void_p()
        dev = (ctypes.c_int * 1)(device)
        _check(lib.shd_ctx_create(dev, 1, ctypes.byref(ctx)))
        _ctx = ctx
    return _ctx


def make_batch(stream, n, ts_ptr, col_ptrs, null_ptrs, mem=SHD_MEM_HOST, call_offsets=None, advance_time=True,
               base_seq=None):
    """An shd_batch over the given pointers, and the ctypes arrays it points
    into (keep them alive until the push returns)."""
    ncols = len(col_ptrs)
    cols = (ctypes.c_void_p * max(ncols, 1))(*col_ptrs)
    nulls = (ctypes.c_void_p * max(ncols, 1))(*null_ptrs)
    b = ShdBatch()
    b.stream = stream
    b.mem = mem
    b.n = n
    b.ts = ts_ptr
    b.ncols = ncols
    b.cols = ctypes.cast(cols, ctypes.c_void_p)
    b.nulls = ctypes.cast(nulls, ctypes.c_void_p)
    co = None
    if call_offsets is not None:
        co = np.ascontiguousarray(call_offsets, np.int64)
        b.ncalls = len(co) - 1
        b.call_offsets = co.ctypes.data
    else:
        b.ncalls = 0
        b.call_offsets = None
    b.advance_time = 1 if advance_time else 0
    if base_seq is not None:
        b.use_base_seq = 1
        b.base_seq = int(base_seq)
    return b, (cols, nulls, co)


class DeviceQuery:
    """Thin owner of one shd_query (used by the engine and by bench.py)."""

    def __init__(self, ir: bytes, device: int = 0):
        self.lib = load_library()
        ctx = context(device)
        self._ir = ctypes.create_string_buffer(ir, len(ir))
        q = ctypes.c_void_p()
        _check(self.lib.shd_plan_load(ctx, self._ir, len(ir), ctypes.byref(q)))
        self.q = q

    @property
    def engine_kind(self) -> int:
        """Engine the query runs on now (a pattern query moves to the generic
        NFA engine when its input leaves the forward scan's formulation)."""
        e = ctypes.c_int()
        _check(self.lib.shd_plan_engine(self.q, ctypes.byref(e)))
        return e.value

    def close(self):
        if self.q:
            self.lib.shd_plan_free(self.q)
            self.q = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push_raw(self, stream, n, ts_ptr, col_ptrs: List[int], null_ptrs: List[int], mem=SHD_MEM_HOST,
                 call_offsets: np.ndarray = None, advance_time=True, base_seq=None):
        """shd_push.  base_seq: arrival index of the first event in the whole
        (sharded) stream, so that in_seq of the rows is global (shd_batch.base_seq)."""
        b, keep = make_batch(stream, n, ts_ptr, col_ptrs, null_ptrs, mem, call_offsets, advance_time, base_seq)
        _check(self.lib.shd_push(self.q, ctypes.byref(b)))

    def set_time(self, t):
        _check(self.lib.shd_set_time(self.q, int(t)))

    def set_option(self, key: str, value: int):
        """shd_set_option: e.g. ("exact_aggregates", 1) = bit-exact sequential
        window folds instead of the default segmented scans."""
        _check(self.lib.shd_set_option(self.q, key.encode(), int(value)))

    def flush(self):
        _check(self.lib.shd_flush(self.q))

    def discard(self):
        _check(self.lib.shd_discard_output(self.q))

    def reset(self):
        _check(self.lib.shd_reset(self.q))

    def poll(self, with_seq=False):
        """Rows since the last poll: (chunk, type, ts, values, nulls), plus in_seq
        (arrival index of the emitting input event, shd_out.in_seq) when with_seq."""
        o = ShdOut()
        _check(self.lib.shd_poll(self.q, ctypes.byref(o)))
        n, nc = o.n_rows, o.n_cols
        if n == 0:
            return None
        chunk = np.ctypeslib.as_array(ctypes.cast(o.chunk, ctypes.POINTER(ctypes.c_int64)), (n,)).copy()
        seq = np.ctypeslib.as_array(ctypes.cast(o.in_seq, ctypes.POINTER(ctypes.c_int64)), (n,)).copy()
        # shd_out.state_idx: state id of the emitting processor, per row
        self.last_state_idx = np.ctypeslib.as_array(ctypes.cast(o.state_idx, ctypes.POINTER(ctypes.c_int32)),
                                                    (n,)).copy()
        nl = o.n_list
        # list arena of OBJECT columns (shd_out.list_values / list_nulls)
        if nl > 0:
            self.last_lists = (
                np.ctypeslib.as_array(ctypes.cast(o.list_values, ctypes.POINTER(ctypes.c_uint64)), (nl,)).copy(),
                np.ctypeslib.as_array(ctypes.cast(o.list_nulls, ctypes.POINTER(ctypes.c_uint8)), (nl,)).copy())
        else:
            self.last_lists = (np.zeros(0, np.uint64), np.zeros(0, np.uint8))
        typ = np.ctypeslib.as_array(ctypes.cast(o.type, ctypes.POINTER(ctypes.c_int32)), (n,)).copy()
        ts = np.ctypeslib.as_array(ctypes.cast(o.ts, ctypes.POINTER(ctypes.c_int64)), (n,)).copy()
        if nc > 0:
            vals = np.ctypeslib.as_array(ctypes.cast(o.values, ctypes.POINTER(ctypes.c_uint64)), (n * nc,)).copy()
            nul = np.ctypeslib.as_array(ctypes.cast(o.nulls, ctypes.POINTER(ctypes.c_uint8)), (n * nc,)).copy()
            vals = vals.reshape(n, nc)
            nul = nul.reshape(n, nc)
        else:
            vals = np.zeros((n, 0), np.uint64)
            nul = np.zeros((n, 0), np.uint8)
        if with_seq:
            return chunk, typ, ts, vals, nul, seq
        return chunk, typ, ts, vals, nul

    def counters(self) -> dict:
        c = ShdCounters()
        _check(self.lib.shd_get_counters(self.q, ctypes.byref(c)))
        return {f: getattr(c, f) for f, _ in ShdCounters._fields_}

    def stage_times(self) -> dict:
        ns = (ctypes.c_int64 * 16)()
        names = (ctypes.c_char_p * 16)()
        n = ctypes.c_int()
        _check(self.lib.shd_stage_times(self.q, ns, names, 16, ctypes.byref(n)))
        return {names[i].decode(): ns[i] for i in range(n.value)}

    def snapshot(self) -> bytes:
        """Device state image (shd_snapshot); pending output must have been polled."""
        data, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.shd_snapshot(self.q, ctypes.byref(data), ctypes.byref(n)))
        return ctypes.string_at(data, n.value)

    def restore(self, image: bytes):
        buf = ctypes.create_string_buffer(image, len(image))
        _check(self.lib.shd_restore(self.q, buf, len(image)))

    def stream_handle(self):
        s = ctypes.c_void_p()
        _check(self.lib.shd_query_stream(self.q, ctypes.byref(s)))
        return s.value


class DeviceGroup:
    """shd_group over fresh member DeviceQuery objects: one forward scan of the
    leader plan (planner.share_pattern_queries) serves every member; poll the
    members as usual.  Close the group before the members."""

    def __init__(self, leader_ir: bytes, members: List[DeviceQuery], device: int = 0):
        self.lib = load_library()
        ctx = context(device)
        self._ir = ctypes.create_string_buffer(leader_ir, len(leader_ir))
        arr = (ctypes.c_void_p * len(members))(*[m.q.value for m in members])
        g = ctypes.c_void_p()
        _check(self.lib.shd_group_create(ctx, self._ir, len(leader_ir), arr, len(members), ctypes.byref(g)))
        self.g = g
        self.members = list(members)

    def push_raw(self, stream, n, ts_ptr, col_ptrs, null_ptrs, mem=SHD_MEM_HOST, call_offsets=None,
                 advance_time=True, base_seq=None):
        b, keep = make_batch(stream, n, ts_ptr, col_ptrs, null_ptrs, mem, call_offsets, advance_time, base_seq)
        _check(self.lib.shd_group_push(self.g, ctypes.byref(b)))

    def reset(self):
        _check(self.lib.shd_group_reset(self.g))

    def _leader(self):
        q = ctypes.c_void_p()
        _check(self.lib.shd_group_leader(self.g, ctypes.byref(q)))
        return q

    def leader_engine_kind(self) -> int:
        e = ctypes.c_int()
        _check(self.lib.shd_plan_engine(self._leader(), ctypes.byref(e)))
        return e.value

    def counters(self) -> dict:
        """The shared scan's counters (the leader query's)."""
        c = ShdCounters()
        _check(self.lib.shd_get_counters(self._leader(), ctypes.byref(c)))
        return {f: getattr(c, f) for f, _ in ShdCounters._fields_}

    def stage_times(self) -> dict:
        ns = (ctypes.c_int64 * 16)()
        names = (ctypes.c_char_p * 16)()
        n = ctypes.c_int()
        _check(self.lib.shd_stage_times(self._leader(), ns, names, 16, ctypes.byref(n)))
        return {names[i].decode(): ns[i] for i in range(n.value)}

    def close(self):
        if self.g:
            self.lib.shd_group_free(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HipQueryEngine:
    """Query engine of SiddhiAppRuntime backed by libsiddhi_hip (MI355X)."""

    # a push may hold several InputHandler calls (shd_batch.call_offsets):
    # the engine advances playback time per call (SiddhiAppRuntime._batch_push_ok)
    batch_calls = True

    def __init__(self, qp: pl.QueryPlan, dictionary, exact_aggregates: bool = False):
        self.qp = qp
        try:
            self.dq = DeviceQuery(qp.ir)
        except SiddhiHipError as e:
            if e.code == SHD_E_UNSUPPORTED:
                raise pl.UnsupportedPlanException(str(e))
            raise
        if exact_aggregates and self.dq.engine_kind == 2:
            self.dq.set_option("exact_aggregates", 1)
        self.types = qp.plan.stream_types

    @property
    def engine_name(self):
        return ENGINE_NAMES.get(self.dq.engine_kind, "?")

    def close(self):
        self.dq.close()

    def _drain(self) -> List[OutputChunk]:
        r = self.dq.poll()
        if r is None:
            return []
        lcols = list_columns(self.qp)
        objs = decode_lists(r[3], lcols, *self.dq.last_lists) if lcols else None
        return split_chunks(*r, objs)

    def start(self, t):
        """SiddhiAppRuntime.start() at app time t (shd_set_option "start_time")."""
        self.dq.set_option("start_time", int(t))

    def set_time(self, t):
        self.dq.set_time(t)
        return self._drain()

    def push(self, si, batch, advance_time=False):
        cols = [np.ascontiguousarray(c) for c in batch.cols]
        nulls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in batch.nulls]
        ts = np.ascontiguousarray(batch.ts, np.int64)
        self.dq.push_raw(si, batch.n, ts.ctypes.data, [c.ctypes.data for c in cols],
                         [0 if x is None else x.ctypes.data for x in nulls], SHD_MEM_HOST,
                         batch.call_offsets if len(batch.call_offsets) > 2 else None, advance_time)
        return self._drain()

    def counters(self):
        return self.dq.counters()

    def snapshot(self) -> bytes:
        return self.dq.snapshot()

    def restore(self, image: bytes):
        self.dq.restore(image)
