"""SiddhiQL subset compiler: app text -> query AST.

Host-side restatement of the parts of the reference grammar that the hot path
uses (`modules/siddhi-query-compiler/src/main/antlr4/io/siddhi/query/compiler/
SiddhiQL.g4`):

* `define stream` (g4 `definition_stream`),
* annotations `@app:playback`, `@app:name`, `@info(name=...)`,
* single-stream queries with filters and `#window.length/time` (g4 :190-192),
* pattern (`->`) and sequence (`,`) inputs with `every`, `within`, count
  `<m:n>` / `* ? +`, logical `and`/`or`, absent `not X for t` (g4 :200-335),
* select / group by / having / insert [current|expired|all events] into
  (g4 :357-426),
* `partition with (attr of Stream, ...) begin ... end` (g4 :154-170).

The AST mirrors the reference query-api object model
(`modules/siddhi-query-api/src/main/java/io/siddhi/query/api/execution/query/
input/state/*StateElement.java`): StreamStateElement, NextStateElement,
EveryStateElement, LogicalStateElement, CountStateElement,
AbsentStreamStateElement.

Associativity of `->`/`,` follows ANTLR4 left recursion (left-assoc); every
binds to the immediately following source or parenthesised chain.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union

# --------------------------------------------------------------------------- types
TYPES = ("string", "int", "long", "float", "double", "bool", "object")


class SiddhiParserException(Exception):
    """Mirrors io.siddhi.query.compiler.exception.SiddhiParserException."""


class OutOfScopeSyntax(SiddhiParserException):
    """Valid SiddhiQL that the hot-path compiler does not cover."""


# --------------------------------------------------------------------------- AST
@dataclass
class Const:
    type: str            # int/long/float/double/bool/string/null
    value: object


@dataclass
class Var:
    attr: str
    stream: Optional[str] = None      # stream id or event reference (e1)
    index: Optional[int] = None       # >=0, or LAST=-2, LAST-1=-3 ... (query-api Variable)


@dataclass
class BinOp:
    op: str                           # + - * / % > < >= <= == != and or
    left: object
    right: object


@dataclass
class Not:
    expr: object


@dataclass
class IsNull:
    expr: object                      # Var or stream reference (StreamRef)


@dataclass
class StreamRef:
    """`e1 is null` form (null_check over a stream_reference)."""
    stream: str
    index: Optional[int] = None


@dataclass
class Func:
    name: str
    args: list
    namespace: Optional[str] = None


@dataclass
class Filter:
    expr: object


@dataclass
class Window:
    name: str
    params: list


@dataclass
class StreamDef:
    name: str
    attrs: List[Tuple[str, str]]
    annotations: list = field(default_factory=list)


@dataclass
class SingleInput:
    stream: str
    handlers: list                   # [Filter|Window] in textual order
    ref: Optional[str] = None
    inner: bool = False


@dataclass
class StreamSE:
    stream: str
    ref: Optional[str]
    filters: List[object]
    absent: bool = False
    waiting_ms: Optional[int] = None


@dataclass
class NextSE:
    a: object
    b: object


@dataclass
class EverySE:
    inner: object


@dataclass
class LogicalSE:
    kind: str                          # 'and' | 'or'
    a: StreamSE
    b: StreamSE


@dataclass
class CountSE:
    stream: StreamSE
    min: int                           # ANY = -1
    max: int                           # ANY = -1


@dataclass
class StateInput:
    kind: str                          # 'pattern' | 'sequence'
    element: object
    within_ms: Optional[int] = None


@dataclass
class OutAttr:
    expr: object
    name: str


@dataclass
class Selector:
    select_all: bool
    attrs: List[OutAttr]
    group_by: List[Var] = field(default_factory=list)
    having: object = None
    order_by: list = field(default_factory=list)
    limit: object = None
    offset: object = None


@dataclass
class OutputRate:
    unit: str       # events | time
    kind: str       # all | first | last | snapshot (time only)
    value: int      # events, or ms


@dataclass
class Query:
    name: Optional[str]
    input: object
    selector: Selector
    target: str
    event_type: str = "current"        # current | expired | all
    annotations: list = field(default_factory=list)
    inner_target: bool = False
    output_rate: object = None


@dataclass
class Partition:
    with_: List[Tuple[object, str]]    # (key expression, stream id)
    queries: List[Query]
    annotations: list = field(default_factory=list)


@dataclass
class Annotation:
    name: str                          # e.g. 'app:playback', 'info'
    elements: List[Tuple[Optional[str], str]]

    def get(self, key, default=None):
        for k, v in self.elements:
            if k is not None and k.lower() == key.lower():
                return v
        return default


@dataclass
class SiddhiApp:
    annotations: List[Annotation]
    streams: dict                      # name -> StreamDef
    queries: List[Query]
    partitions: List[Partition]
    execution_order: list              # Query | Partition in text order

    def annotation(self, name):
        for a in self.annotations:
            if a.name.lower() == name.lower():
                return a
        return None


LAST = -2

# --------------------------------------------------------------------------- lexer
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[fFdDlL]?)
  | (?P<id>`[^`]*`|[A-Za-z_][A-Za-z_0-9]*)
  | (?P<op>->|==|!=|>=|<=|[-+*/%<>=()\[\],;:.#@!?])
""", re.S | re.X)


@dataclass
class Tok:
    kind: str
    text: str
    pos: int

    @property
    def low(self):
        return self.text.lower()


def tokenize(text: str) -> List[Tok]:
    out = []
    i = 0
    while i < len(text):
        m = _TOKEN_RE.match(text, i)
        if not m:
            raise SiddhiParserException("unexpected character %r at %d" % (text[i], i))
        kind = m.lastgroup
        if kind != "ws":
            t = m.group(kind)
            if kind == "id" and t.startswith("`"):
                t = t[1:-1]
            out.append(Tok(kind, t, i))
        i = m.end()
    out.append(Tok("eof", "", len(text)))
    return out


_TIME_UNITS = [
    (re.compile(r"^years?$"), 365 * 24 * 3600 * 1000),
    (re.compile(r"^months?$"), 30 * 24 * 3600 * 1000),
    (re.compile(r"^weeks?$"), 7 * 24 * 3600 * 1000),
    (re.compile(r"^days?$"), 24 * 3600 * 1000),
    (re.compile(r"^hours?$"), 3600 * 1000),
    (re.compile(r"^min(ute|utes)?$"), 60 * 1000),
    (re.compile(r"^sec(ond|onds)?$"), 1000),
    (re.compile(r"^millisec(ond|onds)?$"), 1),
]


def _time_unit(word: str) -> Optional[int]:
    w = word.lower()
    for rx, ms in _TIME_UNITS:
        if rx.match(w):
            return ms
    return None


# --------------------------------------------------------------------------- parser
class Parser:
    def __init__(self, text: str):
        self.toks = tokenize(text)
        self.i = 0

    # -- token helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def at(self, *words, k=0) -> bool:
        t = self.peek(k)
        return t.low in words if t.kind in ("id",) else t.text in words

    def at_kw(self, *words, k=0) -> bool:
        t = self.peek(k)
        return t.kind == "id" and t.low in words

    def accept(self, text) -> bool:
        t = self.peek()
        if (t.kind == "id" and t.low == text) or (t.kind == "op" and t.text == text):
            self.i += 1
            return True
        return False

    def expect(self, text) -> Tok:
        t = self.peek()
        if (t.kind == "id" and t.low == text) or (t.kind == "op" and t.text == text):
            self.i += 1
            return t
        raise SiddhiParserException("expected %r but found %r at %d" % (text, t.text, t.pos))

    def name(self) -> str:
        t = self.next()
        if t.kind != "id":
            raise SiddhiParserException("expected name but found %r at %d" % (t.text, t.pos))
        return t.text

    # -- app
    def parse_app(self) -> SiddhiApp:
        app_ann, streams, queries, partitions, order = [], {}, [], [], []
        pending_ann: List[Annotation] = []
        while self.peek().kind != "eof":
            if self.accept(";"):
                continue
            if self.at("@"):
                ann = self.annotation()
                if ann.name.lower().startswith("app:"):
                    app_ann.append(ann)
                else:
                    pending_ann.append(ann)
                continue
            if self.at_kw("define"):
                sd = self.define_stream()
                sd.annotations = pending_ann
                pending_ann = []
                streams[sd.name] = sd
                continue
            if self.at_kw("from"):
                q = self.query(pending_ann)
                pending_ann = []
                queries.append(q)
                order.append(q)
                continue
            if self.at_kw("partition"):
                p = self.partition(pending_ann)
                pending_ann = []
                partitions.append(p)
                order.append(p)
                continue
            t = self.peek()
            raise SiddhiParserException("unexpected %r at %d" % (t.text, t.pos))
        return SiddhiApp(app_ann, streams, queries, partitions, order)

    def annotation(self) -> Annotation:
        self.expect("@")
        name = self.name()
        while self.accept(":") or self.accept("."):
            name += ":" + self.name()
        elems = []
        if self.accept("("):
            if not self.accept(")"):
                while True:
                    if self.at("@"):
                        self.annotation()   # nested annotations ignored
                    else:
                        key = None
                        if self.peek(1).text == "=" or (self.peek(1).text in (".", ":", "-") and self.peek().kind == "id"):
                            parts = [self.name()]
                            while self.peek().text in (".", ":", "-"):
                                self.next()
                                parts.append(self.name())
                            key = ".".join(parts)
                            self.expect("=")
                        t = self.next()
                        val = t.text[1:-1] if t.kind == "str" else t.text
                        elems.append((key, val))
                    if self.accept(")"):
                        break
                    self.expect(",")
        return Annotation(name, elems)

    def define_stream(self) -> StreamDef:
        self.expect("define")
        kind = self.name().lower()
        if kind != "stream":
            raise SiddhiParserException("only 'define stream' is supported on the hot path, found define %s" % kind)
        name = self.name()
        self.expect("(")
        attrs = []
        while True:
            an = self.name()
            ty = self.name().lower()
            if ty not in TYPES:
                raise SiddhiParserException("unknown attribute type %s" % ty)
            attrs.append((an, ty))
            if self.accept(")"):
                break
            self.expect(",")
        return StreamDef(name, attrs)

    def partition(self, anns) -> Partition:
        self.expect("partition")
        self.expect("with")
        self.expect("(")
        withs = []
        while True:
            e = self.expression()
            if self.at_kw("as"):
                raise OutOfScopeSyntax("range partitions are out of scope")
            self.expect("of")
            sid = self.name()
            withs.append((e, sid))
            if self.accept(")"):
                break
            self.expect(",")
        self.expect("begin")
        qs = []
        pend = []
        while not self.at_kw("end"):
            if self.accept(";"):
                continue
            if self.at("@"):
                pend.append(self.annotation())
                continue
            qs.append(self.query(pend))
            pend = []
        self.expect("end")
        return _inner_streams(Partition(withs, qs, anns))

    # -- query
    def query(self, anns) -> Query:  # noqa: C901
        self.expect("from")
        inp = self.query_input()
        if self.at_kw("select"):
            sel = self.selector()
        else:
            sel = Selector(True, [])
        rate = None
        if self.accept("output"):
            # output_rate (SiddhiQL.g4): output [all|first|last] every <n> events | <time>
            # | output snapshot every <time>
            if self.accept("snapshot"):
                self.expect("every")
                rate = OutputRate("time", "snapshot", self.time_value())
            kind = self.name().lower() if rate is None and self.at_kw("all", "first", "last") else "all"
            if rate is None:
                self.expect("every")
                if self.peek().kind == "num" and self.at_kw("events", "event", k=1):
                    n = int(self.next().text)
                    self.next()
                    rate = OutputRate("events", kind, n)
                else:
                    rate = OutputRate("time", kind, self.time_value())
        self.expect("insert")
        et = "current"
        if self.at_kw("all", "expired", "current", "events"):
            w = self.name().lower()
            if w == "events":
                et = "current"
            else:
                et = w
                self.expect("events")
        self.expect("into")
        inner = self.accept("#")
        target = self.name()
        name = None
        for a in anns:
            if a.name.lower() == "info":
                name = a.get("name")
        return Query(name, inp, sel, target, et, anns, inner, rate)

    def query_input(self):
        # Decide between standard stream, pattern and sequence by scanning to the
        # end of the input section (select / insert at depth 0).
        depth, j = 0, self.i
        saw_arrow = saw_comma = saw_every = saw_eq = saw_not = False
        while True:
            t = self.toks[j]
            if t.kind == "eof":
                break
            if t.text in ("(", "["):
                depth += 1
            elif t.text in (")", "]"):
                depth -= 1
            elif depth == 0 and t.kind == "id" and t.low in ("select", "insert", "output"):
                break
            elif depth == 0 and t.text == "->":
                saw_arrow = True
            elif depth == 0 and t.text == ",":
                saw_comma = True
            elif t.kind == "id" and t.low == "every":
                saw_every = True
            elif t.kind == "id" and t.low == "not" and depth == 0:
                saw_not = True
            elif depth == 0 and t.text == "=" and self.toks[j - 1].kind == "id":
                saw_eq = True
            elif depth == 0 and t.kind == "id" and t.low in ("join", "unidirectional"):
                raise OutOfScopeSyntax("joins are outside the hot path")
            j += 1
        if saw_arrow or (saw_every and not saw_comma) or (saw_not and not saw_comma) or (saw_eq and not saw_comma):
            el = self.pattern_chain()
            within = self.within()
            return StateInput("pattern", el, within)
        if saw_comma:
            el = self.sequence_chain(top=True)
            within = self.within()
            return StateInput("sequence", el, within)
        return self.standard_stream()

    def within(self):
        if self.accept("within"):
            return self.time_value()
        return None

    def time_value(self) -> int:
        total = 0
        seen = False
        while self.peek().kind == "num" and self.peek(1).kind == "id" and _time_unit(self.peek(1).text) is not None:
            n = int(self.next().text)
            total += n * _time_unit(self.next().text)
            seen = True
        if not seen:
            raise SiddhiParserException("expected time value at %d" % self.peek().pos)
        return total

    def standard_stream(self) -> SingleInput:
        inner = self.accept("#")
        sid = ("#" if inner else "") + self.name()
        handlers = []
        while True:
            if self.at("["):
                self.next()
                handlers.append(Filter(self.expression()))
                self.expect("]")
            elif self.at("#") and self.peek(1).kind == "id" and self.peek(1).low == "window":
                self.next(); self.next(); self.expect(".")
                wname = self.name()
                self.expect("(")
                params = []
                if not self.accept(")"):
                    while True:
                        params.append(self.expression())
                        if self.accept(")"):
                            break
                        self.expect(",")
                handlers.append(Window(wname.lower() if ":" not in wname else wname, params))
            elif self.at("#") and self.peek(1).text == "[":
                self.next()
            elif self.at("#"):
                raise OutOfScopeSyntax("stream functions are out of scope for the hot path")
            else:
                break
        ref = None
        if self.accept("as"):
            ref = self.name()
        return SingleInput(sid, handlers, ref, inner)

    # -- patterns (g4 every_pattern_source_chain / pattern_source_chain)
    def pattern_chain(self):
        left = self.pattern_unit()
        while self.accept("->"):
            right = self.pattern_unit()
            left = NextSE(left, right)
        return left

    def pattern_unit(self):
        if self.accept("every"):
            if self.at("(") and not self._paren_is_logical_absent():
                self.next()
                inner = self.pattern_chain()
                self.expect(")")
                return EverySE(inner)
            return EverySE(self.pattern_source())
        if self.at("(") and not self._paren_is_logical_absent():
            self.next()
            inner = self.pattern_chain()
            self.expect(")")
            return inner
        return self.pattern_source()

    def _paren_is_logical_absent(self):
        # '(' not X and e=Y ')' style logical absent sources are parsed by pattern_source
        return self.peek(1).kind == "id" and self.peek(1).low == "not"

    def pattern_source(self, sequence=False):
        """logical | collection | standard | absent (g4 pattern_source / sequence_source)."""
        if self.at("(") and self._paren_is_logical_absent():
            self.next()
            s = self.pattern_source(sequence)
            self.expect(")")
            return s
        a = self.stateful_or_absent()
        if self.at_kw("and", "or"):
            kind = self.name().lower()
            b = self.stateful_or_absent()
            if b.absent and not a.absent:
                # the absent operand of a mixed pair is element 1 (SiddhiQLBaseVisitorImpl.
                # visitLogical_absent_stateful_source -> State.logicalNotAnd / logicalOr(absent, present))
                a, b = b, a
            return LogicalSE(kind, a, b)
        if isinstance(a, StreamSE) and not a.absent:
            if self.at("<"):
                self.next()
                mn, mx = self.collect()
                self.expect(">")
                return CountSE(a, mn, mx)
            if sequence and self.peek().text in ("*", "?", "+"):
                t = self.next().text
                return CountSE(a, {"*": 0, "?": 0, "+": 1}[t], {"*": -1, "?": 1, "+": -1}[t])
        return a

    def collect(self):
        if self.accept(":"):
            return -1, int(self.next().text)
        a = int(self.next().text)
        if self.accept(":"):
            if self.peek().kind == "num":
                return a, int(self.next().text)
            return a, -1
        return a, a

    def stateful_or_absent(self) -> StreamSE:
        if self.accept("not"):
            sid, filters = self.basic_source()
            waiting = None
            if self.accept("for"):
                waiting = self.time_value()
            return StreamSE(sid, None, filters, True, waiting)
        ref = None
        if self.peek().kind == "id" and self.peek(1).text == "=":
            ref = self.name()
            self.expect("=")
        sid, filters = self.basic_source()
        return StreamSE(sid, ref, filters)

    def basic_source(self):
        # `#Name`: a partition-inner stream (rewritten by _inner_streams)
        sid = ("#" + self.name()) if self.accept("#") else self.name()
        filters = []
        while self.at("[") or (self.at("#") and self.peek(1).text == "["):
            self.accept("#")
            self.expect("[")
            filters.append(self.expression())
            self.expect("]")
        if self.at("#"):
            raise OutOfScopeSyntax("stream functions inside patterns are out of scope")
        return sid, filters

    # -- sequences (g4 every_sequence_source_chain)
    def sequence_chain(self, top=False):
        left = self.sequence_unit(first=top)
        while self.accept(","):
            right = self.sequence_unit(first=False)
            left = NextSE(left, right)
        return left

    def sequence_unit(self, first=False):
        if first and self.accept("every"):
            return EverySE(self.sequence_unit(False))
        if self.at("(") and not self._paren_is_logical_absent():
            self.next()
            inner = self.sequence_chain()
            self.expect(")")
            return inner
        return self.pattern_source(sequence=True)

    # -- selector
    def selector(self) -> Selector:
        self.expect("select")
        if self.accept("*"):
            sel = Selector(True, [])
        else:
            attrs = []
            while True:
                e = self.expression()
                if self.accept("as"):
                    nm = self.name()
                elif isinstance(e, Var):
                    nm = e.attr
                else:
                    raise SiddhiParserException("select expression needs 'as <name>'")
                attrs.append(OutAttr(e, nm))
                if not self.accept(","):
                    break
            sel = Selector(False, attrs)
        if self.accept("group"):
            self.expect("by")
            while True:
                v = self.primary()
                if not isinstance(v, Var):
                    raise SiddhiParserException("group by needs attribute references")
                sel.group_by.append(v)
                if not self.accept(","):
                    break
        if self.accept("having"):
            sel.having = self.expression()
        if self.at_kw("order", "limit", "offset"):
            raise OutOfScopeSyntax("order by / limit / offset are out of scope for the hot path")
        return sel

    # -- expressions (g4 math_operation precedence)
    def expression(self):
        return self.or_expr()

    def or_expr(self):
        l = self.and_expr()
        while self.at_kw("or") and not self._logical_source_ahead():
            self.next()
            l = BinOp("or", l, self.and_expr())
        return l

    def and_expr(self):
        l = self.eq_expr()
        while self.at_kw("and") and not self._logical_source_ahead():
            self.next()
            l = BinOp("and", l, self.eq_expr())
        return l

    def _logical_source_ahead(self):
        return False

    def eq_expr(self):
        l = self.rel_expr()
        while self.peek().text in ("==", "!="):
            op = self.next().text
            l = BinOp(op, l, self.rel_expr())
        return l

    def rel_expr(self):
        l = self.add_expr()
        while self.peek().text in (">", "<", ">=", "<="):
            op = self.next().text
            l = BinOp(op, l, self.add_expr())
        return l

    def add_expr(self):
        l = self.mul_expr()
        while self.peek().text in ("+", "-"):
            op = self.next().text
            l = BinOp(op, l, self.mul_expr())
        return l

    def mul_expr(self):
        l = self.unary()
        while self.peek().text in ("*", "/", "%"):
            op = self.next().text
            l = BinOp(op, l, self.unary())
        return l

    def unary(self):
        if self.at_kw("not"):
            self.next()
            return Not(self.unary())
        if self.peek().text in ("-", "+") and self.peek(1).kind == "num":
            sign = self.next().text
            c = self.number()
            if sign == "-":
                c = Const(c.type, -c.value)
            return c
        return self.primary()

    def number(self) -> Const:
        t = self.next()
        # time constants: "10 sec"
        if self.peek().kind == "id" and _time_unit(self.peek().text) is not None and re.fullmatch(r"\d+", t.text):
            self.i -= 1
            return Const("long", self.time_value())
        s = t.text
        low = s.lower()
        if low.endswith("l"):
            return Const("long", int(s[:-1]))
        if low.endswith("f"):
            return Const("float", float(s[:-1]))
        if low.endswith("d"):
            return Const("double", float(s[:-1]))
        if re.fullmatch(r"\d+", s):
            v = int(s)
            return Const("int", v)
        return Const("double", float(s))

    def primary(self):
        t = self.peek()
        if t.text == "(":
            self.next()
            e = self.expression()
            self.expect(")")
            return self._maybe_is_null(e)
        if t.kind == "num":
            return self.number()
        if t.kind == "str":
            self.next()
            return Const("string", t.text[1:-1])
        if t.kind == "id" and t.low in ("true", "false") and self.peek(1).text not in ("(", ".", "["):
            self.next()
            return Const("bool", t.low == "true")
        if t.kind == "id" and t.low == "null" and self.peek(1).text not in ("(", "."):
            self.next()
            return Const("null", None)
        if t.text == "#" or t.text == "!":
            self.next()
        if t.kind == "id" or t.text in ("#", "!"):
            nm = self.name()
            # function call (namespace:fn(...) or fn(...))
            if self.at(":") and self.peek(1).kind == "id" and self.peek(2).text == "(":
                self.next()
                fn = self.name()
                return self._maybe_is_null(self._call(fn, nm))
            if self.at("("):
                return self._maybe_is_null(self._call(nm, None))
            index = None
            if self.at("["):
                self.next()
                if self.accept("last"):
                    index = LAST
                    if self.accept("-"):
                        index = LAST - int(self.next().text)
                else:
                    index = int(self.next().text)
                self.expect("]")
            if self.accept("."):
                attr = self.name()
                return self._maybe_is_null(Var(attr, nm, index))
            if index is not None:
                if self.at_kw("is"):
                    return self._maybe_is_null(StreamRef(nm, index))
                raise SiddhiParserException("stream index without attribute at %d" % t.pos)
            if self.at_kw("is") and self.peek(1).kind == "id" and self.peek(1).low == "null":
                # could be attribute or stream reference; resolved by the planner
                return self._maybe_is_null(Var(nm))
            return Var(nm)
        raise SiddhiParserException("unexpected %r at %d" % (t.text, t.pos))

    def _call(self, fn, ns):
        self.expect("(")
        args = []
        if not self.accept(")"):
            if self.accept("*"):
                self.expect(")")
            else:
                while True:
                    args.append(self.expression())
                    if self.accept(")"):
                        break
                    self.expect(",")
        return Func(fn, args, ns)

    def _maybe_is_null(self, e):
        if self.at_kw("is") and self.peek(1).kind == "id" and self.peek(1).low == "null":
            self.next(); self.next()
            return IsNull(e)
        return e


def parse(app_text: str) -> SiddhiApp:
    """SiddhiCompiler.parse equivalent (QC/java/io/siddhi/query/compiler/SiddhiCompiler.java)."""
    return Parser(app_text).parse_app()


# ---------------------------------------------------------------- partition-inner streams
def _qualify(expr, ref):
    """A partition key expression over a stream's attributes, read through
    the pattern state `ref` (e1.quantity)."""
    if isinstance(expr, Var):
        return Var(expr.attr, ref if expr.stream is None else expr.stream, expr.index)
    if isinstance(expr, BinOp):
        return BinOp(expr.op, _qualify(expr.left, ref), _qualify(expr.right, ref))
    if isinstance(expr, Not):
        return Not(_qualify(expr.expr, ref))
    return expr


def _state_streams(el):
    """StreamSE leaves of a pattern / sequence element in text order."""
    if isinstance(el, StreamSE):
        return [el]
    if isinstance(el, NextSE):
        return _state_streams(el.a) + _state_streams(el.b)
    if isinstance(el, EverySE):
        return _state_streams(el.inner)
    if isinstance(el, LogicalSE):
        return [el.a, el.b]
    if isinstance(el, CountSE):
        return [el.stream]
    if isinstance(el, (list, tuple)):
        return [x for e in el for x in _state_streams(e)]
    return []


PKEY = "__pkey"


def _inner_streams(p: Partition) -> Partition:
    """`insert into #S` / `from #S` inside a partition (PartitionRuntimeImpl:
    an inner stream is per partition instance, C/partition/
    PartitionRuntimeImpl.java:346-402): the producer's rows carry the key of
    the instance that emitted them as a hidden attribute `__pkey` (its input
    stream's partition key, read through the first keyed pattern state), and
    the inner stream joins the partition keyed by it -- so a consumer's
    per-key state sees exactly the rows its own instance produced."""
    keys = {sid: e for e, sid in p.with_}
    inner = {q.target for q in p.queries if q.inner_target}
    if not inner:
        return p
    for q in p.queries:
        if not q.inner_target:
            continue
        if q.selector.select_all:
            raise OutOfScopeSyntax("select * into a partition-inner stream is outside the hot path")
        inp = q.input
        if isinstance(inp, SingleInput):
            k = keys.get(inp.stream)
            kexpr = None if k is None else (_qualify(k, inp.ref) if inp.ref else k)
        elif isinstance(inp, StateInput):
            kexpr = None
            for se in _state_streams(inp.element):
                if not se.absent and se.ref is not None and se.stream in keys:
                    kexpr = _qualify(keys[se.stream], se.ref)
                    break
        else:
            kexpr = None
        if kexpr is None:
            raise OutOfScopeSyntax("partition-inner stream '%s' from a query without a keyed input" % q.target)
        q.selector.attrs.append(OutAttr(kexpr, PKEY))
        q.target = "#" + q.target
        q.inner_target = False
    for q in p.queries:
        if isinstance(q.input, SingleInput) and q.input.inner:
            q.input.inner = False
    p.with_ = list(p.with_) + [(Var(PKEY), "#" + n) for n in sorted(inner)]
    return p
