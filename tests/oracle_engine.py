"""Query engine backed by the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE: used only as the checker in tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg.  The product
(siddhi_amd) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

from siddhi_amd import planner as pl
from siddhi_amd.runtime import OutputChunk, decode_lists, list_columns, split_chunks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def load_oracle():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ROOT, "oracle", "oracle.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(LIB)
    P = ctypes.c_void_p
    lib.orc_create.restype = P
    lib.orc_create.argtypes = [P, ctypes.c_int64]
    lib.orc_destroy.argtypes = [P]
    lib.orc_push.restype = ctypes.c_int
    lib.orc_push.argtypes = [P, ctypes.c_int32, ctypes.c_int64, P, P, P, ctypes.c_int32]
    lib.orc_set_time.restype = ctypes.c_int
    lib.orc_set_time.argtypes = [P, ctypes.c_int64]
    lib.orc_start.restype = ctypes.c_int
    lib.orc_start.argtypes = [P, ctypes.c_int64]
    lib.orc_num_rows.restype = ctypes.c_int64
    lib.orc_num_rows.argtypes = [P]
    lib.orc_num_outputs.restype = ctypes.c_int32
    lib.orc_num_outputs.argtypes = [P]
    lib.orc_get_rows.argtypes = [P, P, P, P, P, P]
    lib.orc_clear_rows.argtypes = [P]
    lib.orc_get_rows_seq.argtypes = [P, P]
    lib.orc_num_list.restype = ctypes.c_int64
    lib.orc_num_list.argtypes = [P]
    lib.orc_get_list.argtypes = [P, P, P]
    lib.orc_counters.argtypes = [P, P]
    lib.orc_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def to_bits(col: np.ndarray, t: int) -> np.ndarray:
    if t == pl.T_INT:
        return col.astype(np.int64).view(np.uint64)
    if t == pl.T_LONG:
        return col.astype(np.int64).view(np.uint64)
    if t == pl.T_FLOAT:
        return col.astype(np.float32).view(np.uint32).astype(np.uint64)
    if t == pl.T_DOUBLE:
        return col.astype(np.float64).view(np.uint64)
    return col.astype(np.uint64)


class OracleQueryEngine:
    def __init__(self, qp: pl.QueryPlan, dictionary):
        self.lib = load_oracle()
        self.qp = qp
        words = np.frombuffer(qp.ir, np.int32).copy()
        self._ir = words
        self.h = self.lib.orc_create(words.ctypes.data, len(words))
        if not self.h:
            raise pl.SiddhiAppCreationException("oracle: " + self.lib.orc_last_error().decode())
        self.n_out = self.lib.orc_num_outputs(self.h)
        self.types = qp.plan.stream_types
        self._log = []
        self.drained_seq = []

    def close(self):
        if self.h:
            self.lib.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _drain(self):
        n = self.lib.orc_num_rows(self.h)
        if n == 0:
            return []
        chunk = np.empty(n, np.int64)
        typ = np.empty(n, np.int32)
        ts = np.empty(n, np.int64)
        vals = np.empty((n, max(self.n_out, 1)), np.uint64)
        nul = np.empty((n, max(self.n_out, 1)), np.uint8)
        self.lib.orc_get_rows(self.h, chunk.ctypes.data, typ.ctypes.data, ts.ctypes.data,
                              vals.ctypes.data, nul.ctypes.data)
        sq = np.empty(n, np.int64)
        self.lib.orc_get_rows_seq(self.h, sq.ctypes.data)
        self.drained_seq.append(sq)   # shd_out.in_seq of the drained rows
        nl = self.lib.orc_num_list(self.h)
        lv = np.zeros(max(nl, 1), np.uint64)
        ln = np.zeros(max(nl, 1), np.uint8)
        if nl:
            self.lib.orc_get_list(self.h, lv.ctypes.data, ln.ctypes.data)
        self.last_lists = (lv, ln)
        self.lib.orc_clear_rows(self.h)
        lcols = list_columns(self.qp)
        objs = decode_lists(vals, lcols, lv, ln) if lcols else None
        return split_chunks(chunk, typ, ts, vals[:, :self.n_out], nul[:, :self.n_out], objs)

    # snapshot / restore for the checker: the oracle's state is a function of
    # its input history, so its "snapshot" is that history (replayed into a
    # fresh oracle on restore).  Serialized with numpy (no pickle).
    def snapshot(self) -> bytes:
        import io
        arrs = {}
        for i, op in enumerate(self._log):
            if op[0] == "t":
                arrs["op%d_t" % i] = np.array([op[1]], np.int64)
            elif op[0] == "s":
                arrs["op%d_s" % i] = np.array([op[1]], np.int64)
            else:
                _, si, b, adv = op
                arrs["op%d_p" % i] = np.array([si, 1 if adv else 0, len(b.cols)], np.int64)
                arrs["op%d_ts" % i] = np.asarray(b.ts, np.int64)
                arrs["op%d_co" % i] = np.asarray(b.call_offsets, np.int64)
                for a, c in enumerate(b.cols):
                    arrs["op%d_c%d" % (i, a)] = np.asarray(c)
                    if b.nulls[a] is not None:
                        arrs["op%d_n%d" % (i, a)] = np.asarray(b.nulls[a], np.uint8)
        bio = io.BytesIO()
        np.savez(bio, n_ops=np.array([len(self._log)], np.int64), **arrs)
        return bio.getvalue()

    def restore(self, image: bytes):
        import io
        from siddhi_amd.runtime import ColumnBatch
        z = np.load(io.BytesIO(image), allow_pickle=False)
        self.close()
        words = self._ir
        self.h = self.lib.orc_create(words.ctypes.data, len(words))
        self._log = []
        for i in range(int(z["n_ops"][0])):
            if "op%d_t" % i in z:
                self.set_time(int(z["op%d_t" % i][0]))
                continue
            if "op%d_s" % i in z:
                self.start(int(z["op%d_s" % i][0]))
                continue
            si, adv, nc = (int(x) for x in z["op%d_p" % i])
            cols = [z["op%d_c%d" % (i, a)] for a in range(nc)]
            nulls = [z["op%d_n%d" % (i, a)] if ("op%d_n%d" % (i, a)) in z else None for a in range(nc)]
            self.push(si, ColumnBatch(z["op%d_ts" % i], cols, nulls, z["op%d_co" % i]), bool(adv))

    def start(self, t):
        """SiddhiAppRuntime.start() at app time t."""
        self._log.append(("s", int(t)))
        if self.lib.orc_start(self.h, int(t)) != 0:
            raise RuntimeError("oracle: " + self.lib.orc_last_error().decode())

    def set_time(self, t):
        self._log.append(("t", int(t)))
        if self.lib.orc_set_time(self.h, int(t)) != 0:
            raise RuntimeError("oracle: " + self.lib.orc_last_error().decode())
        return self._drain()

    def push(self, si, batch, advance_time=False):
        self._log.append(("p", si, batch, advance_time))
        types = self.types[si]
        n = batch.n
        vals = np.empty((n, max(len(types), 1)), np.uint64)
        nul = np.zeros((n, max(len(types), 1)), np.uint8)
        for a, t in enumerate(types):
            vals[:, a] = to_bits(batch.cols[a], t)
            if batch.nulls[a] is not None:
                nul[:, a] = batch.nulls[a]
        vals = np.ascontiguousarray(vals[:, :len(types)]) if types else vals
        nul = np.ascontiguousarray(nul[:, :len(types)]) if types else nul
        ts = np.ascontiguousarray(batch.ts, np.int64)
        if self.lib.orc_push(self.h, si, n, ts.ctypes.data, vals.ctypes.data, nul.ctypes.data,
                             1 if advance_time else 0) != 0:
            raise RuntimeError("oracle: " + self.lib.orc_last_error().decode())
        return self._drain()

    def counters(self):
        c = np.zeros(8, np.int64)
        self.lib.orc_counters(self.h, c.ctypes.data)
        return c
