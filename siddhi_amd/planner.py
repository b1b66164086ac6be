"""Planner: query AST -> typed plan IR (include/siddhi_ir.h).

Restates the reference planning rules the hot path depends on:

* state ids in parse order, logical element 2 before element 1
  (C/util/parser/StateInputStreamParser.java:148-408),
* variable resolution incl. the `[last]` rule inside a state's own filter
  (C/util/parser/ExpressionParser.java:1254-1439, :1262-1263, :1378-1385),
  default chain index CURRENT for filters (SingleInputStreamParser.java:185-188)
  and 0 for the selector (SelectorParser.java:215-218),
* arithmetic result type = widest of DOUBLE > FLOAT > LONG > INT
  (ExpressionParser.java:1488-1506),
* compare promotion per executor class (C/executor/condition/compare/*):
  relational ops use Java binary promotion; == / != on (Float, Long) or
  (Long, Float) compare as double,
* aggregator return types (SumAttributeAggregatorExecutor.java:84-134: INT/LONG
  -> LONG, FLOAT/DOUBLE -> DOUBLE; avg -> DOUBLE; count -> LONG).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import query_compiler as qc

# ---- IR constants (mirror include/siddhi_ir.h) -----------------------------
MAGIC, VERSION = 0x50444853, 1
POST_MAGIC = 0x54534F50
KIND_STATE, KIND_SINGLE = 1, 2
T_STRING, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL = 0, 1, 2, 3, 4, 5
T_OBJECT = 6   # output only: a list over a count state's chain (include/siddhi_ir.h SHD_T_OBJECT)
TYPE_CODE = {"string": T_STRING, "int": T_INT, "long": T_LONG, "float": T_FLOAT,
             "double": T_DOUBLE, "bool": T_BOOL}
TYPE_NAME = {v: k for k, v in TYPE_CODE.items()}
TYPE_NAME[T_OBJECT] = "object"
(OP_END, OP_CONST, OP_NULL, OP_LOAD, OP_EVNULL, OP_CVT, OP_ADD, OP_SUB, OP_MUL,
 OP_DIV, OP_MOD, OP_EQ, OP_NE, OP_GT, OP_GE, OP_LT, OP_LE, OP_AND, OP_OR, OP_NOT,
 OP_ISNULL, OP_AGG, OP_TS, OP_IFELSE, OP_MULTI) = range(25)
IDX_CURRENT, IDX_LAST = -1, -2
NODE_STREAM, NODE_NEXT, NODE_EVERY, NODE_LOGICAL, NODE_COUNT = 1, 2, 3, 4, 5
H_FILTER, H_WINDOW = 1, 2
W_LENGTH, W_TIME, W_LENGTH_BATCH, W_TIME_BATCH, W_TIME_LENGTH, W_EXTERNAL_TIME = 1, 2, 3, 4, 5, 6
W_TIME_BATCH_STREAM = 7
INT64_MIN = -(1 << 63)
AGG_SUM, AGG_AVG, AGG_COUNT = 1, 2, 3
UNKNOWN_STATE = -1
NUMERIC_RANK = {T_INT: 0, T_LONG: 1, T_FLOAT: 2, T_DOUBLE: 3}
ARITH_OPS = {"+": OP_ADD, "-": OP_SUB, "*": OP_MUL, "/": OP_DIV, "%": OP_MOD}
CMP_OPS = {"==": OP_EQ, "!=": OP_NE, ">": OP_GT, ">=": OP_GE, "<": OP_LT, "<=": OP_LE}


class SiddhiAppCreationException(Exception):
    """Mirrors io.siddhi.core.exception.SiddhiAppCreationException."""


class SiddhiAppValidationException(SiddhiAppCreationException):
    """Mirrors io.siddhi.query.api.exception.SiddhiAppValidationException."""


class UnsupportedPlanException(SiddhiAppCreationException):
    """The plan is valid SiddhiQL but outside the MI355X hot path (SHD_E_UNSUPPORTED)."""


# ---- string dictionary -----------------------------------------------------
class StringDictionary:
    """Host dictionary: string -> u32 id. Only equality is used on strings in
    the hot path (SURVEY.md §7 'Dictionary-encoding strings')."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.strings: List[str] = []

    def id(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.strings)
            self.ids[s] = i
            self.strings.append(s)
        return i

    def lookup(self, i: int) -> str:
        return self.strings[i]


# ---- plan model --------------------------------------------------------------
@dataclass
class Meta:
    ref: Optional[str]
    stream: str
    attrs: List[Tuple[str, int]]      # (name, type code)
    multi: bool = False

    def attr(self, name):
        for i, (n, t) in enumerate(self.attrs):
            if n == name:
                return i, t
        return None


@dataclass
class Plan:
    kind: int
    query_name: Optional[str]
    streams: List[str]                          # plan stream index -> app stream id
    stream_types: List[List[int]]
    consts: List[int] = field(default_factory=list)
    exprs: List[List[Tuple[int, int, int, int]]] = field(default_factory=list)
    partition_keys: List[Tuple[int, int]] = field(default_factory=list)   # (stream, expr)
    # state
    state_type: int = 0
    within: int = -1
    n_states: int = 0
    tree: List[int] = field(default_factory=list)
    # single
    single_stream: int = 0
    handlers: List[Tuple] = field(default_factory=list)
    # selector
    current_on: bool = True
    expired_on: bool = False
    aggs: List[Tuple[int, int, int]] = field(default_factory=list)        # (kind, expr, arg type)
    group_by: List[int] = field(default_factory=list)
    having: int = -1
    outputs: List[Tuple[str, int, int]] = field(default_factory=list)     # (name, type, expr)
    # dictionary id of the string "null": a null string group-by value builds
    # the same group key as the string "null" (GroupByKeyGenerator appends
    # String.valueOf(null), C/query/selector/GroupByKeyGenerator.java:63-73);
    # -1 when no group-by attribute is a string.  Optional trailing IR words.
    null_str_id: int = -1
    # STATE plans with an aggregating / `having` selector: (base outputs
    # [(type, expr)], nested SINGLE plan) -- the IR's POST section
    post: Optional[Tuple[List[Tuple[int, int]], "Plan"]] = None
    target: str = ""
    # descriptive (host/runtime only)
    states: List[Meta] = field(default_factory=list)
    shape: Dict = field(default_factory=dict)

    # -- serialization
    def to_words(self) -> List[int]:
        w = [MAGIC, VERSION, self.kind, len(self.streams)]
        for types in self.stream_types:
            w.append(len(types))
            w.extend(types)
        w.append(len(self.consts))
        for c in self.consts:
            c &= (1 << 64) - 1
            w.append(_s32(c & 0xFFFFFFFF))
            w.append(_s32(c >> 32))
        w.append(len(self.exprs))
        for e in self.exprs:
            w.append(len(e))
            for ins in e:
                w.extend(ins)
        w.append(len(self.partition_keys))
        for s, e in self.partition_keys:
            w.extend([s, e])
        if self.kind == KIND_STATE:
            w.extend([self.state_type, *_split64(self.within), self.n_states])
            w.extend(self.tree)
        else:
            w.extend([self.single_stream, len(self.handlers)])
            for h in self.handlers:
                if h[0] == H_FILTER:
                    w.extend([H_FILTER, h[1]])
                else:
                    w.extend([H_WINDOW, h[1], *_split64(h[2]), *_split64(h[3] if len(h) > 3 else 0)])
        w.extend([int(self.current_on), int(self.expired_on), len(self.aggs)])
        for a in self.aggs:
            w.extend(a)
        w.append(len(self.group_by))
        w.extend(self.group_by)
        w.append(self.having)
        w.append(len(self.outputs))
        for _, t, e in self.outputs:
            w.extend([t, e])
        w.extend(_split64(self.null_str_id))
        if self.post is not None:
            base, sub = self.post
            sw = sub.to_words()
            w.extend([POST_MAGIC, len(base)])
            for t, e in base:
                w.extend([t, e])
            w.append(len(sw))
            w.extend(sw)
        return w

    def to_bytes(self) -> bytes:
        words = self.to_words()
        return struct.pack("<%di" % len(words), *words)


def _s32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _split64(v):
    v &= (1 << 64) - 1
    return _s32(v & 0xFFFFFFFF), _s32(v >> 32)


def const_bits(type_code: int, value) -> int:
    """64-bit payload of a value of the given type (see include/siddhi_ir.h)."""
    if type_code in (T_INT, T_LONG):
        return int(value) & ((1 << 64) - 1)
    if type_code == T_FLOAT:
        return struct.unpack("<I", struct.pack("<f", float(value)))[0]
    if type_code == T_DOUBLE:
        return struct.unpack("<Q", struct.pack("<d", float(value)))[0]
    if type_code == T_BOOL:
        return 1 if value else 0
    if type_code == T_STRING:
        return int(value)
    raise ValueError(type_code)


# ---- expression compiler -------------------------------------------------------
class ExprCompiler:
    def __init__(self, plan: Plan, dictionary: StringDictionary, metas: List[Meta],
                 state_query: bool):
        self.plan = plan
        self.dict = dictionary
        self.metas = metas
        self.state_query = state_query
        self.agg_allowed = False
        self.multi_top = None

    def compile(self, expr, current_state: int, default_index: int, want_bool=False,
                allow_agg=False, allow_multi=False) -> Tuple[int, int]:
        """Returns (expr id, result type).  allow_multi: a selector output that
        is one variable may be a multi-value selection (SHD_OP_MULTI)."""
        code: List[Tuple[int, int, int, int]] = []
        self.agg_allowed = allow_agg
        self.multi_top = expr if allow_multi and isinstance(expr, qc.Var) else None
        t = self._emit(expr, code, current_state, default_index)
        if want_bool and t != T_BOOL:
            raise SiddhiAppValidationException("condition must be of type BOOL but found %s" % TYPE_NAME.get(t))
        self.plan.exprs.append(code)
        return len(self.plan.exprs) - 1, t

    def _const(self, t, v):
        bits = const_bits(t, v)
        try:
            idx = self.plan.consts.index(bits)
        except ValueError:
            self.plan.consts.append(bits)
            idx = len(self.plan.consts) - 1
        return idx

    def _emit(self, e, code, cs, di) -> int:
        if isinstance(e, qc.Const):
            if e.type == "null":
                code.append((OP_NULL, 0, T_DOUBLE, 0))
                return T_DOUBLE
            t = TYPE_CODE[e.type]
            v = self.dict.id(e.value) if t == T_STRING else e.value
            code.append((OP_CONST, self._const(t, v), t, 0))
            return t
        if isinstance(e, qc.Var):
            if self.state_query and e.stream is not None and e.attr is not None and \
                    self._is_stream_ref_only(e):
                pass
            return self._emit_var(e, code, cs, di)
        if isinstance(e, qc.IsNull):
            inner = e.expr
            if isinstance(inner, qc.StreamRef) or (isinstance(inner, qc.Var) and inner.stream is None
                                                   and self._ref_state(inner.attr) is not None
                                                   and not self._attr_exists(inner.attr, cs)):
                ref = inner.stream if isinstance(inner, qc.StreamRef) else inner.attr
                idx = inner.index if isinstance(inner, qc.StreamRef) else None
                st = self._ref_state(ref)
                if st is None:
                    raise SiddhiAppValidationException("stream reference %s not found" % ref)
                ci = di if idx is None else (idx + 1 if idx <= qc.LAST else idx)
                code.append((OP_EVNULL, st, ci, 0))
                return T_BOOL
            self._emit(inner, code, cs, di)
            code.append((OP_ISNULL, 0, 0, 0))
            return T_BOOL
        if isinstance(e, qc.Not):
            t = self._emit(e.expr, code, cs, di)
            if t != T_BOOL:
                raise SiddhiAppValidationException("not requires a BOOL operand")
            code.append((OP_NOT, 0, 0, 0))
            return T_BOOL
        if isinstance(e, qc.BinOp):
            if e.op in ("and", "or"):
                lt = self._emit(e.left, code, cs, di)
                rt = self._emit(e.right, code, cs, di)
                if lt != T_BOOL or rt != T_BOOL:
                    raise SiddhiAppValidationException("%s requires BOOL operands" % e.op)
                code.append((OP_AND if e.op == "and" else OP_OR, 0, 0, 0))
                return T_BOOL
            if e.op in ARITH_OPS:
                lcode, rcode = [], []
                lt = self._emit(e.left, lcode, cs, di)
                rt = self._emit(e.right, rcode, cs, di)
                if lt not in NUMERIC_RANK or rt not in NUMERIC_RANK:
                    raise SiddhiAppValidationException("arithmetic on non-numeric operands")
                rtype = max(lt, rt, key=lambda x: NUMERIC_RANK[x])
                code.extend(lcode)
                if lt != rtype:
                    code.append((OP_CVT, lt, rtype, 0))
                code.extend(rcode)
                if rt != rtype:
                    code.append((OP_CVT, rt, rtype, 0))
                code.append((ARITH_OPS[e.op], rtype, 0, 0))
                return rtype
            if e.op in CMP_OPS:
                lcode, rcode = [], []
                lt = self._emit(e.left, lcode, cs, di)
                rt = self._emit(e.right, rcode, cs, di)
                ct = compare_type(e.op, lt, rt)
                code.extend(lcode)
                if lt != ct:
                    code.append((OP_CVT, lt, ct, 0))
                code.extend(rcode)
                if rt != ct:
                    code.append((OP_CVT, rt, ct, 0))
                code.append((CMP_OPS[e.op], ct, 0, 0))
                return T_BOOL
            raise SiddhiAppValidationException("unknown operator %s" % e.op)
        if isinstance(e, qc.Func):
            name = e.name.lower()
            if e.namespace is None and name in ("sum", "avg", "count"):
                if not self.agg_allowed:
                    raise SiddhiAppValidationException("aggregator %s not allowed here" % name)
                if name == "count":
                    arg, at = -1, -1
                    if e.args:
                        # count(attr) counts events regardless of nulls
                        arg, at = ExprCompiler(self.plan, self.dict, self.metas, self.state_query) \
                            .compile(e.args[0], cs, di)
                    self.plan.aggs.append((AGG_COUNT, arg, at))
                    rt = T_LONG
                else:
                    if len(e.args) != 1:
                        raise SiddhiAppValidationException("%s needs exactly one parameter" % name)
                    sub = ExprCompiler(self.plan, self.dict, self.metas, self.state_query)
                    arg, at = sub.compile(e.args[0], cs, di)
                    if at not in NUMERIC_RANK:
                        raise SiddhiAppValidationException("%s not supported for %s" % (name, TYPE_NAME.get(at)))
                    self.plan.aggs.append((AGG_SUM if name == "sum" else AGG_AVG, arg, at))
                    rt = (T_LONG if at in (T_INT, T_LONG) else T_DOUBLE) if name == "sum" else T_DOUBLE
                code.append((OP_AGG, len(self.plan.aggs) - 1, 0, 0))
                return rt
            if e.namespace is None and name == "eventtimestamp" and not e.args:
                code.append((OP_TS, 0, IDX_CURRENT, 0))
                return T_LONG
            if e.namespace is None and name == "ifthenelse":
                # IfThenElseFunctionExecutor (C/executor/function/IfThenElseFunctionExecutor.java):
                # all three arguments are evaluated, a true condition picks the
                # second, anything else (false, null) the third
                if len(e.args) != 3:
                    raise SiddhiAppValidationException("Invalid no of arguments passed to ifThenElse() function, "
                                                       "required only 3, but found %d" % len(e.args))
                if self._emit(e.args[0], code, cs, di) != T_BOOL:
                    raise SiddhiAppValidationException("Input type of if in ifThenElse function should be of "
                                                       "type BOOL")
                t1 = self._emit(e.args[1], code, cs, di)
                t2 = self._emit(e.args[2], code, cs, di)
                if t1 != t2:
                    raise SiddhiAppValidationException("Input type of then in ifThenElse function and else in "
                                                       "ifThenElse function should be of equivalent type")
                code.append((OP_IFELSE, t1, 0, 0))
                return t1
            if e.namespace is None and name in _INSTANCE_OF:
                # InstanceOf*FunctionExecutor (C/executor/function/InstanceOf*.java):
                # `data instanceof X`; an attribute's value is boxed as its
                # declared type, so the test is "non-null" for that type and
                # false for every other
                if len(e.args) != 1:
                    raise SiddhiAppValidationException("Invalid no of arguments passed to %s() function" % e.name)
                scratch: List[Tuple[int, int, int, int]] = []
                t = self._emit(e.args[0], scratch, cs, di)
                if t == _INSTANCE_OF[name]:
                    code.extend(scratch)
                    code.append((OP_ISNULL, 0, 0, 0))
                    code.append((OP_NOT, 0, 0, 0))
                else:
                    code.append((OP_CONST, self._const(T_BOOL, False), T_BOOL, 0))
                return T_BOOL
            raise UnsupportedPlanException("function %s is outside the hot path" % e.name)
        raise SiddhiAppValidationException("unsupported expression %r" % (e,))

    def _is_stream_ref_only(self, e):
        return False

    def _ref_state(self, ref):
        for i, m in enumerate(self.metas):
            if m.ref == ref or (m.ref is None and m.stream == ref):
                return i
        return None

    def _attr_exists(self, attr, cs):
        if cs >= 0:
            return self.metas[cs].attr(attr) is not None
        return any(m.attr(attr) is not None for m in self.metas)

    def _emit_var(self, v: qc.Var, code, cs, di) -> int:
        """ExpressionParser.parseVariable (C/util/parser/ExpressionParser.java:1254-1439)."""
        if v.index is not None:
            ci = v.index + 1 if v.index <= qc.LAST else v.index
        else:
            ci = di
        if not self.state_query:
            m = self.metas[0]
            if v.stream is not None and v.stream != m.stream and v.stream != m.ref:
                raise SiddhiAppValidationException("Id '%s' not defined within the current scope" % v.stream)
            found = m.attr(v.attr)
            if found is None:
                raise SiddhiAppValidationException("No matching stream reference found for attribute '%s'" % v.attr)
            code.append((OP_LOAD, 0, IDX_CURRENT, found[0] | (found[1] << 16)))
            return found[1]
        state, typ, attr = None, None, None
        if v.stream is None:
            if cs == UNKNOWN_STATE:
                for i, m in enumerate(self.metas):
                    f = m.attr(v.attr)
                    if f is not None:
                        if state is not None:
                            raise SiddhiAppValidationException(
                                "Input streams contain attribute with same name '%s'" % v.attr)
                        state, (attr, typ) = i, f
            else:
                f = self.metas[cs].attr(v.attr)
                if f is None:
                    raise SiddhiAppValidationException("attribute '%s' not found in state %d" % (v.attr, cs))
                state, (attr, typ) = cs, f
        else:
            for i, m in enumerate(self.metas):
                if m.ref is None:
                    if m.stream == v.stream:
                        f = m.attr(v.attr)
                        if f is None:
                            raise SiddhiAppValidationException("attribute %s not in %s" % (v.attr, m.stream))
                        state, (attr, typ) = i, f
                        break
                elif m.ref == v.stream:
                    f = m.attr(v.attr)
                    if f is None:
                        raise SiddhiAppValidationException("attribute %s not in %s" % (v.attr, m.stream))
                    state, (attr, typ) = i, f
                    if cs > -1 and self.metas[cs].ref is not None and v.index is not None \
                            and v.index <= qc.LAST and v.stream == self.metas[cs].ref:
                        ci = v.index
                    elif cs == UNKNOWN_STATE and v.index is None and m.multi:
                        # ExpressionParser.parseVariable (:1386-1388, :1430-1437): a count
                        # state's attribute without an index in the selector is the
                        # MultiValueVariableFunctionExecutor -- a List of the attribute
                        # over the whole chain (type OBJECT)
                        if self.multi_top is not v:
                            raise UnsupportedPlanException(
                                "multi-value selection of count state '%s' inside an expression" % v.stream)
                        code.append((OP_MULTI, i, 0, f[0] | (f[1] << 16)))
                        return T_OBJECT
                    break
        if state is None:
            if v.stream is None:
                raise SiddhiAppValidationException(
                    "No matching stream reference found for attribute '%s'" % v.attr)
            raise SiddhiAppValidationException(
                "Stream with reference '%s' not found for attribute '%s'" % (v.stream, v.attr))
        code.append((OP_LOAD, state, ci, attr | (typ << 16)))
        return typ


def compare_type(op, lt, rt) -> int:
    """Operand type each compare executor class compares in
    (C/executor/condition/compare/*/*CompareConditionExpressionExecutor*.java)."""
    if lt == T_STRING or rt == T_STRING:
        if lt == rt == T_STRING and op in ("==", "!="):
            return T_STRING
        raise SiddhiAppValidationException("string comparison %s not supported" % op)
    if lt == T_BOOL or rt == T_BOOL:
        if lt == rt == T_BOOL and op in ("==", "!="):
            return T_BOOL
        raise SiddhiAppValidationException("bool comparison %s not supported" % op)
    if op in ("==", "!=") and {lt, rt} == {T_FLOAT, T_LONG}:
        return T_DOUBLE
    return max(lt, rt, key=lambda x: NUMERIC_RANK[x])


# ---- query planning -------------------------------------------------------------
@dataclass
class QueryPlan:
    plan: Plan
    ir: bytes
    input_streams: List[str]
    output_names: List[str]
    output_types: List[int]
    target: str
    name: Optional[str]
    partitioned: bool
    receiver_kind: Dict[str, str]        # stream -> 'single' | 'multi' (state queries)
    # `output ... every` (C/query/output/ratelimit/**): applied by the host runtime
    # to the selector's output chunks; rate_group_cols: the output columns that
    # hold the group-by values (GroupedComplexEvent keys)
    output_rate: Optional[object] = None
    rate_group_cols: Optional[List[int]] = None


def _stream_meta(app: qc.SiddhiApp, sid: str, ref=None, extra_streams=None) -> Meta:
    sd = app.streams.get(sid) or (extra_streams or {}).get(sid)
    if sd is None:
        raise SiddhiAppValidationException("Stream '%s' is not defined" % sid)
    return Meta(ref, sid, [(n, TYPE_CODE[t]) for n, t in sd.attrs])


def plan_query(app: qc.SiddhiApp, q: qc.Query, dictionary: StringDictionary,
               partition: Optional[qc.Partition] = None, extra_streams=None) -> QueryPlan:
    inp = q.input
    if q.inner_target or getattr(inp, "inner", False) or _uses_inner_stream(inp):
        raise UnsupportedPlanException("partition-inner streams (#stream) are outside the hot path")
    if isinstance(inp, qc.StateInput):
        qp = _plan_state(app, q, dictionary, partition, extra_streams)
    elif isinstance(inp, qc.SingleInput):
        qp = _plan_single(app, q, dictionary, partition, extra_streams)
    else:
        raise UnsupportedPlanException("input kind %s is outside the hot path" % type(inp).__name__)
    if q.output_rate is not None:
        _plan_output_rate(qp, q, partition)
    return qp


def _plan_output_rate(qp: QueryPlan, q: qc.Query, partition):
    """Output rate limiting (OutputParser.constructOutputRateLimiter,
    C/util/parser/OutputParser.java:282-331): event- and time-based, all / first
    / last, per group when the query groups.  Its state is per partition key
    inside a partition (refused here); a group's key is its group-by values,
    which must be selected as they are."""
    if partition is not None:
        raise UnsupportedPlanException("output rate limiting inside a partition is outside the hot path")
    rate = q.output_rate
    if rate.value <= 0:
        raise SiddhiAppValidationException("output rate should be positive")
    if rate.kind == "snapshot":
        # WrappedSnapshotOutputRateLimiter.init (C/query/output/ratelimit/
        # snapshot/WrappedSnapshotOutputRateLimiter.java:67-115): a windowed
        # input picks the window-content limiters (they track what the window
        # holds), the rest PerSnapshot / GroupByPerSnapshot.  QueryParser
        # disables the selector's batching for all of them (QueryParser.java:
        # 217-223): an aggregating selector then emits one row per event where
        # this runtime's engines emit one per call and group, so only
        # non-windowed, non-aggregating queries are exact here.
        if isinstance(q.input, qc.SingleInput) and any(isinstance(h, qc.Window) for h in q.input.handlers):
            raise UnsupportedPlanException("output snapshot on a windowed input (the windowed snapshot limiters) "
                                           "is outside the hot path")
        if q.selector and any(_has_agg(oa.expr) for oa in q.selector.attrs):
            raise UnsupportedPlanException("output snapshot with aggregations (per-event selector output) is "
                                           "outside the hot path")
    qp.output_rate = rate
    gb = q.selector.group_by if q.selector else []
    if gb and rate.kind in ("first", "last", "snapshot"):
        cols = []
        for g in gb:
            hit = None
            for c, oa in enumerate(q.selector.attrs):
                if isinstance(oa.expr, qc.Var) and oa.expr.attr == g.attr and oa.expr.index is None and \
                        (g.stream is None or oa.expr.stream in (None, g.stream)):
                    hit = c
                    break
            if hit is None and q.selector.select_all and g.attr in qp.output_names:
                hit = qp.output_names.index(g.attr)
            if hit is None:
                raise UnsupportedPlanException("output %s every ... with group by needs the group-by attributes "
                                               "selected as they are" % rate.kind)
            cols.append(hit)
        qp.rate_group_cols = cols


def _plan_partition(plan: Plan, comp_factory, partition, streams: List[str], app, dictionary,
                    extra_streams):
    if partition is None:
        return
    for kexpr, sid in partition.with_:
        if sid not in streams:
            continue
        si = streams.index(sid)
        m = _stream_meta(app, sid, None, extra_streams)
        ec = ExprCompiler(plan, dictionary, [m], state_query=False)
        eid, t = ec.compile(kexpr, 0, IDX_CURRENT)
        plan.partition_keys.append((si, eid))
    missing = [s for s in streams if s not in [sid for _, sid in partition.with_]]
    if missing:
        raise UnsupportedPlanException("partition without a key for streams %s (broadcast) is outside the hot path"
                                       % missing)


def _plan_selector(plan: Plan, q: qc.Query, ec: ExprCompiler, metas: List[Meta], state_query: bool):
    sel = q.selector
    plan.current_on = q.event_type in ("current", "all")
    plan.expired_on = q.event_type in ("expired", "all")
    names, types = [], []
    if sel.select_all:
        if state_query:
            attrs = []
            for st, m in enumerate(metas):
                for (n, t) in m.attrs:
                    attrs.append(qc.OutAttr(qc.Var(n, m.ref or m.stream, None), n))
        else:
            attrs = [qc.OutAttr(qc.Var(n), n) for n, _ in metas[0].attrs]
    else:
        attrs = sel.attrs
    cs = UNKNOWN_STATE if state_query else 0
    for oa in attrs:
        eid, t = ec.compile(oa.expr, cs, 0, allow_agg=True, allow_multi=state_query)
        plan.outputs.append((oa.name, t, eid))
        names.append(oa.name)
        types.append(t)
    for g in sel.group_by:
        eid, gt = ec.compile(g, cs, 0)
        plan.group_by.append(eid)
        if gt == T_STRING:
            plan.null_str_id = ec.dict.id("null")
    if sel.having is not None:
        # QuerySelector's having condition is parsed against the selector's
        # output event (SelectorParser.parse, C/util/parser/SelectorParser.java:
        # havingConditionExecutor over the output attributes): an attribute name
        # of the select list stands for that output's expression
        outs = {oa.name: oa.expr for oa in attrs}
        hexpr = _subst_outputs(sel.having, outs)
        eid, t = ec.compile(hexpr, cs, 0, allow_agg=True)
        if t != T_BOOL:
            raise SiddhiAppValidationException("having condition must be of type BOOL")
        plan.having = eid
    return names, types


_AGG_FUNCS = ("sum", "avg", "count")
_INSTANCE_OF = {"instanceofboolean": T_BOOL, "instanceofdouble": T_DOUBLE, "instanceoffloat": T_FLOAT,
                "instanceofinteger": T_INT, "instanceoflong": T_LONG, "instanceofstring": T_STRING}


def _has_agg(e) -> bool:
    if isinstance(e, qc.Func):
        if e.namespace is None and e.name.lower() in _AGG_FUNCS:
            return True
        return any(_has_agg(a) for a in e.args)
    if isinstance(e, qc.BinOp):
        return _has_agg(e.left) or _has_agg(e.right)
    if isinstance(e, (qc.Not, qc.IsNull)):
        return _has_agg(e.expr)
    return False


def _reads_event(e) -> bool:
    """Whether an expression reads the StateEvent (a variable, a stream
    reference or eventTimestamp())."""
    if isinstance(e, (qc.Var, qc.StreamRef)):
        return True
    if isinstance(e, qc.Func):
        if e.namespace is None and e.name.lower() == "eventtimestamp":
            return True
        return any(_reads_event(a) for a in e.args)
    if isinstance(e, qc.BinOp):
        return _reads_event(e.left) or _reads_event(e.right)
    if isinstance(e, (qc.Not, qc.IsNull)):
        return _reads_event(e.expr)
    return False


def _lift_bases(e, bases: Dict[str, Tuple[int, object]]):
    """The selector AST with every maximal aggregator-free subtree that reads
    the StateEvent replaced by a base attribute `_b<k>` (bases: repr -> (k, subtree))."""
    if not _has_agg(e):
        if not _reads_event(e):
            return e
        k = bases.setdefault(repr(e), (len(bases), e))[0]
        return qc.Var("_b%d" % k)
    if isinstance(e, qc.Func):
        return qc.Func(e.name, [_lift_bases(a, bases) for a in e.args], e.namespace)
    if isinstance(e, qc.BinOp):
        return qc.BinOp(e.op, _lift_bases(e.left, bases), _lift_bases(e.right, bases))
    if isinstance(e, qc.Not):
        return qc.Not(_lift_bases(e.expr, bases))
    if isinstance(e, qc.IsNull):
        return qc.IsNull(_lift_bases(e.expr, bases))
    return e


def _plan_post_selector(app, q: qc.Query, ec: ExprCompiler, metas: List[Meta], dictionary):
    """Device decomposition of a state query's aggregating / `having`
    selector (include/siddhi_ir.h POST section).  The reference runs
    QuerySelector on a chunk of ONE StateEvent (StateMultiProcessStreamReceiver.
    processAndClear, C/query/input/StateMultiProcessStreamReceiver.java:47-68;
    SingleProcessStreamReceiver.java:48-72), so processInBatchNoGroupBy /
    processInBatchGroupBy (QuerySelector.java:271-373) emit that event whenever
    `having` passes, with the aggregators folded over every earlier match in
    emission order.  The state variables the selector reads become base
    outputs of the state plan; the same selector over a stream of those base
    values is a SINGLE plan (one InputHandler call per match row)."""
    sel = q.selector
    if sel.select_all:
        attrs = [qc.OutAttr(qc.Var(n, m.ref or m.stream, None), n) for m in metas for (n, _) in m.attrs]
    else:
        attrs = sel.attrs
    bases: Dict[str, Tuple[int, object]] = {}
    new_attrs = [qc.OutAttr(_lift_bases(oa.expr, bases), oa.name) for oa in attrs]
    new_group = [_lift_bases(g, bases) for g in sel.group_by]
    new_having = None
    if sel.having is not None:
        new_having = _lift_bases(_subst_outputs(sel.having, {oa.name: oa.expr for oa in attrs}), bases)
    base_out: List[Tuple[int, int]] = []
    base_attrs = []
    for key, (k, node) in sorted(bases.items(), key=lambda kv: kv[1][0]):
        eid, t = ec.compile(node, UNKNOWN_STATE, 0)
        base_out.append((t, eid))
        base_attrs.append(("_b%d" % k, TYPE_NAME[t]))
    sd = qc.StreamDef("_post", base_attrs)
    q2 = qc.Query(q.name, qc.SingleInput("_post", []),
                  qc.Selector(False, new_attrs, new_group, new_having), q.target, q.event_type)
    sub = _plan_single(app, q2, dictionary, None, {"_post": sd})
    return base_out, sub.plan


def _subst_outputs(e, outs):
    """Having AST with unqualified names of the select list replaced by their expressions."""
    if isinstance(e, qc.Var):
        if e.stream is None and e.index is None and e.attr in outs:
            return outs[e.attr]
        return e
    if isinstance(e, qc.BinOp):
        return qc.BinOp(e.op, _subst_outputs(e.left, outs), _subst_outputs(e.right, outs))
    if isinstance(e, qc.Not):
        return qc.Not(_subst_outputs(e.expr, outs))
    if isinstance(e, qc.IsNull):
        return qc.IsNull(_subst_outputs(e.expr, outs))
    if isinstance(e, qc.Func):
        return qc.Func(e.name, [_subst_outputs(a, outs) for a in e.args], e.namespace)
    return e


def _plan_state(app, q, dictionary, partition, extra_streams) -> QueryPlan:
    si: qc.StateInput = q.input
    streams: List[str] = []
    counts: Dict[str, int] = {}
    metas: List[Meta] = []
    plan = Plan(KIND_STATE, q.name, streams, [])
    plan.state_type = 0 if si.kind == "pattern" else 1
    plan.within = si.within_ms if si.within_ms is not None else -1
    ec = ExprCompiler(plan, dictionary, metas, state_query=True)

    def stream_idx(sid):
        if sid not in streams:
            streams.append(sid)
            plan.stream_types.append([t for _, t in _stream_meta(app, sid, None, extra_streams).attrs])
        counts[sid] = counts.get(sid, 0) + 1
        return streams.index(sid)

    def walk(el, multi=False):
        if isinstance(el, qc.StreamSE):
            sidx = stream_idx(el.stream)
            m = _stream_meta(app, el.stream, el.ref, extra_streams)
            m.multi = multi
            metas.append(m)
            state_id = len(metas) - 1
            fids = []
            for f in el.filters:
                eid, _ = ec.compile(f, state_id, IDX_CURRENT, want_bool=True)
                fids.append(eid)
            wait = el.waiting_ms if el.waiting_ms is not None else -1
            return [NODE_STREAM, state_id, sidx, int(el.absent), *_split64(wait), len(fids), *fids]
        if isinstance(el, qc.NextSE):
            a = walk(el.a)
            b = walk(el.b)
            return [NODE_NEXT] + a + b
        if isinstance(el, qc.EverySE):
            return [NODE_EVERY] + walk(el.inner)
        if isinstance(el, qc.LogicalSE):
            b = walk(el.b)       # element 2 first (StateInputStreamParser.java:349-361)
            a = walk(el.a)
            return [NODE_LOGICAL, 0 if el.kind == "and" else 1] + a + b
        if isinstance(el, qc.CountSE):
            inner = walk(el.stream, multi=True)
            return [NODE_COUNT, el.min, el.max] + inner
        raise UnsupportedPlanException("state element %r" % (el,))

    plan.tree = walk(si.element)
    plan.n_states = len(metas)
    plan.states = metas
    names, types = _plan_selector(plan, q, ec, metas, True)
    if plan.aggs or plan.group_by or plan.having >= 0:
        if partition is not None and (plan.aggs or plan.group_by):
            raise UnsupportedPlanException("aggregation over partitioned pattern / sequence output "
                                           "(aggregator state per partition key) is outside the hot path")
        plan.post = _plan_post_selector(app, q, ec, metas, dictionary)
    _plan_partition(plan, None, partition, streams, app, dictionary, extra_streams)
    plan.target = q.target
    plan.shape = classify_state_shape(plan, si)
    recv = {s: ("multi" if counts[s] > 1 else "single") for s in streams}
    return QueryPlan(plan, plan.to_bytes(), list(streams), names, types, q.target, q.name,
                     partition is not None, recv)


def _plan_single(app, q, dictionary, partition, extra_streams) -> QueryPlan:
    si: qc.SingleInput = q.input
    m = _stream_meta(app, si.stream, si.ref, extra_streams)
    plan = Plan(KIND_SINGLE, q.name, [si.stream], [[t for _, t in m.attrs]])
    ec = ExprCompiler(plan, dictionary, [m], state_query=False)
    n_windows = 0
    for h in si.handlers:
        if isinstance(h, qc.Filter):
            if any(x[0] == H_WINDOW and x[1] in (W_LENGTH_BATCH, W_TIME_BATCH, W_TIME_BATCH_STREAM)
                   for x in plan.handlers):
                raise UnsupportedPlanException("a filter after a batch window is outside the hot path")
            eid, _ = ec.compile(h.expr, 0, IDX_CURRENT, want_bool=True)
            plan.handlers.append((H_FILTER, eid))
        else:
            n_windows += 1
            if n_windows > 1:
                raise SiddhiAppValidationException("only one window per stream")
            plan.handlers.append(_window_handler(h, partition is not None, m, si.stream))
    names, types = _plan_selector(plan, q, ec, [m], False)
    _plan_partition(plan, None, partition, [si.stream], app, dictionary, extra_streams)
    plan.target = q.target
    plan.shape = {"kind": "single", "window": next((h[1] for h in plan.handlers if h[0] == H_WINDOW), 0)}
    return QueryPlan(plan, plan.to_bytes(), [si.stream], names, types, q.target, q.name,
                     partition is not None, {si.stream: "single"})


def _window_handler(h, partitioned: bool, meta=None, stream=None):
    """(H_WINDOW, kind, p, q) of a `#window.<name>(...)` handler (include/siddhi_ir.h
    shd_window).  Batch windows in both modes: full batch (expired + RESET +
    current per flush) and `stream.current.event` true (W_TIME_BATCH_STREAM,
    lengthBatch with q = 1: the current events go out as they arrive).
    Refused: `timeBatch` inside a partition (its nextEmitTime is a field of
    the processor shared by every partition key,
    TimeBatchWindowProcessor.java:136,283-300)."""
    ps = h.params

    def const(i, types, what):
        if i >= len(ps) or not isinstance(ps[i], qc.Const) or ps[i].type not in types:
            raise SiddhiAppValidationException("%s window's %s should be a constant %s" %
                                               (h.name, what, "/".join(types)))
        return ps[i].value

    if h.name in ("length", "time"):
        if len(ps) != 1:
            raise SiddhiAppValidationException("%s window needs one constant int/long parameter" % h.name)
        return (H_WINDOW, W_LENGTH if h.name == "length" else W_TIME, int(const(0, ("int", "long"), "parameter")), 0)
    if h.name == "lengthbatch":
        if not 1 <= len(ps) <= 2:
            raise SiddhiAppValidationException("LengthBatch window should have one or two parameters")
        n = int(const(0, ("int",), "window.length"))
        stream_cur = len(ps) == 2 and bool(const(1, ("bool",), "stream.current.event"))
        if n < 0:
            raise SiddhiAppValidationException("LengthBatch window's window.length should not be negative")
        return (H_WINDOW, W_LENGTH_BATCH, n, 1 if stream_cur else 0)
    if h.name == "timebatch":
        if not 1 <= len(ps) <= 3:
            raise SiddhiAppValidationException("TimeBatch window should have one to three parameters")
        t = int(const(0, ("int", "long"), "window.time"))
        start = INT64_MIN
        stream_cur = False
        if len(ps) >= 2:
            if ps[1].type == "bool" and len(ps) == 2:
                stream_cur = bool(ps[1].value)
            else:
                start = int(const(1, ("int", "long"), "start.time"))
                if len(ps) == 3:
                    stream_cur = bool(const(2, ("bool",), "stream.current.event"))
        if partitioned:
            raise UnsupportedPlanException("timeBatch inside a partition is outside the hot path")
        if t <= 0:
            raise SiddhiAppValidationException("TimeBatch window's window.time should be positive")
        return (H_WINDOW, W_TIME_BATCH_STREAM if stream_cur else W_TIME_BATCH, t, start)
    if h.name == "timelength":
        if len(ps) != 2:
            raise SiddhiAppValidationException("TimeLength window should only have two parameters")
        t = int(const(0, ("int", "long"), "window.time"))
        n = int(const(1, ("int",), "window.length"))
        return (H_WINDOW, W_TIME_LENGTH, t, n)
    if h.name == "externaltime":
        if len(ps) != 2:
            raise SiddhiAppValidationException("ExternalTime window should only have two parameters")
        v = ps[0]
        if not isinstance(v, qc.Var) or v.index is not None or v.stream not in (None, stream, meta.ref):
            raise SiddhiAppValidationException("ExternalTime window's timeStamp should be a stream attribute")
        names = [a for a, _ in meta.attrs]
        if v.attr not in names or dict(meta.attrs)[v.attr] != T_LONG:
            raise SiddhiAppValidationException("ExternalTime window's timeStamp should be type long")
        t = int(const(1, ("int", "long"), "window.time"))
        return (H_WINDOW, W_EXTERNAL_TIME, t, names.index(v.attr))
    raise UnsupportedPlanException("window %s is outside the hot path" % h.name)


def _uses_inner_stream(inp) -> bool:
    return False


def classify_state_shape(plan: Plan, si: qc.StateInput) -> Dict:
    """Shape facts the device planner uses to pick kernels (e.g. the 2-state
    `every e1 -> e2 within W` fast path)."""
    el = si.element
    shape = {"kind": "state", "type": si.kind}
    if si.kind == "pattern" and isinstance(el, qc.NextSE) and isinstance(el.a, qc.EverySE) \
            and isinstance(el.a.inner, qc.StreamSE) and isinstance(el.b, qc.StreamSE) \
            and not el.a.inner.absent and not el.b.absent:
        shape["every_a_then_b"] = True
    return shape


# ---------------------------------------------------------------- query sharing
# Queries on one StreamJunction (C/stream/StreamJunction.java:146-272) of the
# form `every e1=A[f1] -> e2=B[f2] within W` that differ only in f1 (and in
# their names / targets) share one forward scan on the device (shd_group_*,
# include/siddhi_hip.h): the leader plan's e1 filter accepts every event any
# member's does, and each member keeps the leader's matches whose e1 passes
# its own f1.

def _e1_site(q: qc.Query):
    """The e1 StreamSE of an `every e1=A[..] -> e2=B[..]` pattern query, else None."""
    si = q.input
    if not isinstance(si, qc.StateInput) or si.kind != "pattern":
        return None
    el = si.element
    if not isinstance(el, qc.NextSE) or not isinstance(el.b, qc.StreamSE) or not isinstance(el.a, qc.EverySE):
        return None
    a = el.a.inner
    if not isinstance(a, qc.StreamSE) or a.absent or el.b.absent:
        return None
    return a


def _length_window(q: qc.Query):
    """The Window handler of a `from S[..]#window.length(L) ... group by` query, else None."""
    si = q.input
    if not isinstance(si, qc.SingleInput) or not q.selector.group_by or q.event_type != "current":
        return None
    wins = [h for h in si.handlers if isinstance(h, qc.Window)]
    if len(wins) != 1 or wins[0].name != "length" or len(wins[0].params) != 1:
        return None
    if not isinstance(wins[0].params[0], qc.Const) or wins[0].params[0].type not in ("int", "long"):
        return None
    return wins[0]


def share_signature(q: qc.Query) -> Optional[str]:
    """Equal for two queries iff they can share one device pass (None: not
    shareable): patterns that differ at most in the e1 filter, or length-window
    group-by aggregates that differ at most in the window length -- beyond the
    query name, annotations and the insert target."""
    if q.output_rate is not None:
        return None
    sel = q.selector
    if isinstance(q.input, qc.StateInput) and (sel.group_by or sel.having is not None or
                                               any(_has_agg(oa.expr) for oa in sel.attrs)):
        return None   # aggregating / having selectors over state output run per query (IR POST section)
    import copy
    if _e1_site(q) is not None:
        q2 = copy.deepcopy(q)
        q2.name, q2.target, q2.annotations = None, "", []
        _e1_site(q2).filters = []
        return "pattern:" + repr(q2)
    if _length_window(q) is not None:
        q2 = copy.deepcopy(q)
        q2.name, q2.target, q2.annotations = None, "", []
        _length_window(q2).params = []
        return "window:" + repr(q2)
    return None


_NUMERIC = ("int", "long", "float", "double")


def _threshold(fs):
    """(op, var, const) when the filter list is one `attr op constant` with op in > >= < <=."""
    if len(fs) != 1:
        return None
    f = fs[0]
    if (isinstance(f, qc.BinOp) and f.op in (">", ">=", "<", "<=") and isinstance(f.left, qc.Var)
            and f.left.index is None and isinstance(f.right, qc.Const) and f.right.type in _NUMERIC):
        return f.op, f.left, f.right
    return None


def leader_e1_filters(filter_lists: List[list]) -> list:
    """e1 filters accepting every event any of the lists accepts: one bound
    when all are `attr > c` (or >=, <, <=) on the same attribute, else the
    disjunction of each member's conjunction."""
    if any(len(fs) == 0 for fs in filter_lists):
        return []
    th = [_threshold(fs) for fs in filter_lists]
    if all(t is not None for t in th) and len({(t[0], repr(t[1])) for t in th}) == 1:
        op = th[0][0]
        pick = min if op in (">", ">=") else max
        c = pick((t[2] for t in th), key=lambda k: k.value)
        return [qc.BinOp(op, th[0][1], c)]
    conj = []
    for fs in filter_lists:
        e = fs[0]
        for f in fs[1:]:
            e = qc.BinOp("and", e, f)
        conj.append(e)
    e = conj[0]
    for c in conj[1:]:
        e = qc.BinOp("or", e, c)
    return [e]


def share_groups(queries: List[qc.Query], max_members: int = 64) -> List[List[int]]:
    """Indices of shareable queries, grouped (>= 2 members, at most max_members each)."""
    by: Dict[str, List[int]] = {}
    for i, q in enumerate(queries):
        sig = share_signature(q)
        if sig is not None:
            by.setdefault(sig, []).append(i)
    out = []
    for idx in by.values():
        for k in range(0, len(idx), max_members):
            part = idx[k:k + max_members]
            if len(part) >= 2:
                out.append(part)
    return out


def plan_shared_leader(app: qc.SiddhiApp, members: List[qc.Query], dictionary: StringDictionary,
                       partition: Optional[qc.Partition] = None) -> QueryPlan:
    """The leader plan of a group of shareable queries (share_groups): for
    patterns, the members' query with the disjunction of their e1 filters;
    for length windows, the member with the longest window (its items cover
    every member's window)."""
    import copy
    sigs = {share_signature(q) for q in members}
    if len(sigs) != 1 or None in sigs:
        raise UnsupportedPlanException("queries differ beyond the e1 filter / window length: not shareable")
    if next(iter(sigs)).startswith("window:"):
        lead = copy.deepcopy(max(members, key=lambda q: int(_length_window(q).params[0].value)))
    else:
        lead = copy.deepcopy(members[0])
        _e1_site(lead).filters = leader_e1_filters([_e1_site(q).filters for q in members])
    lead.name = "shared(%s)" % ",".join(str(q.name) for q in members)
    return plan_query(app, lead, dictionary, partition)
