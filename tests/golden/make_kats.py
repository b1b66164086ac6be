"""Generate known-answer fixtures (tests/golden/kat/*.json) from the reference's
own end-to-end tests.

Reads the reference TestNG sources as text (study only; nothing is executed)
and extracts, per @Test method with a straight-line shape:

* the SiddhiQL app string (concatenated string literals),
* the callback target (QueryCallback query name or StreamCallback stream),
* the InputHandler sends in order, with timestamps: explicit `send(ts, ...)`
  values, or for wall-clock sends a synthetic clock advanced by the
  `Thread.sleep(n)` calls between them (events are spaced 1 ms apart),
* the expected output rows (`assertArrayEquals(new Object[]{...}, ...)`,
  in `case N:` order) and the expected event count.

Only the extracted data (app text, inputs, expected outputs, source
file:line) is written; no Java is copied.  Re-run with
    python tests/golden/make_kats.py
when the reference is mounted at /root/reference.
"""
import json
import os
import re
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/"
FILES = [
    "query/pattern/EveryPatternTestCase.java",
    "query/pattern/CountPatternTestCase.java",
    "query/pattern/LogicalPatternTestCase.java",
    "query/pattern/WithinPatternTestCase.java",
    "query/pattern/ComplexPatternTestCase.java",
    "query/pattern/PatternTestCase.java",
    "query/sequence/SequenceTestCase.java",
    "query/partition/PatternPartitionTestCase.java",
    "query/partition/SequencePartitionTestCase.java",
    "query/partition/WindowPartitionTestCase.java",
    "query/window/LengthWindowTestCase.java",
    "query/window/TimeWindowTestCase.java",
    "query/window/LengthBatchWindowTestCase.java",
    "query/window/TimeBatchWindowTestCase.java",
    "query/window/TimeLengthWindowTestCase.java",
    "query/window/ExternalTimeWindowTestCase.java",
    "query/ratelimit/EventOutputRateLimitTestCase.java",
    "query/ratelimit/TimeOutputRateLimitTestCase.java",
    "query/GroupByTestCase.java",
    "query/FilterTestCase1.java",
    "query/FilterTestCase2.java",
    "query/pattern/absent/AbsentPatternTestCase.java",
    "query/pattern/absent/AbsentWithEveryPatternTestCase.java",
    "query/pattern/absent/EveryAbsentPatternTestCase.java",
    "query/pattern/absent/LogicalAbsentPatternTestCase.java",
    "managment/PlaybackTestCase.java",
]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat")
T0 = 1_500_000_000_000


def split_methods(text):
    out = []
    for m in re.finditer(r"@Test(\([^)]*\))?\s*public void (\w+)\(\)[^{]*\{", text):
        start = m.end()
        depth, i = 1, start
        while depth and i < len(text):
            c = text[i]
            if c == '"':
                j = i + 1
                while text[j] != '"':
                    j += 2 if text[j] == "\\" else 1
                i = j
            elif c == "{":
                depth += 1
            elif c == "}":
                depth -= 1
            i += 1
        line = text.count("\n", 0, m.start()) + 1
        out.append((m.group(2), text[start:i - 1], line, m.group(1) or ""))
    return out


STR_LIT = r'"(?:[^"\\]|\\.)*"'


def java_str(lit):
    return bytes(lit[1:-1], "utf-8").decode("unicode_escape")


def eval_concat(expr, strings):
    parts = []
    for tok in re.finditer(STR_LIT + r"|\w+", expr):
        t = tok.group(0)
        if t.startswith('"'):
            parts.append(java_str(t))
        elif t in strings:
            parts.append(strings[t])
        else:
            raise ValueError("unknown string part %s" % t)
    return "".join(parts)


def parse_values(body):
    """Java literals inside new Object[]{...} -> JSON values (typed tags)."""
    vals = []
    depth = 0
    cur = ""
    items = []
    for c in body:
        if c == "," and depth == 0:
            items.append(cur)
            cur = ""
            continue
        if c in "({":
            depth += 1
        elif c in ")}":
            depth -= 1
        cur += c
    if cur.strip():
        items.append(cur)
    for it in items:
        s = it.strip()
        if s.startswith('"'):
            vals.append(java_str(s))
        elif s == "null":
            vals.append(None)
        elif s in ("true", "false"):
            vals.append(s == "true")
        elif re.fullmatch(r"-?\d+[lL]", s):
            vals.append({"long": int(s[:-1])})
        elif re.fullmatch(r"-?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?[fF]", s):
            vals.append({"float": float(s[:-1])})
        elif re.fullmatch(r"-?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?[dD]?", s) and ("." in s or "e" in s.lower() or s[-1] in "dD"):
            vals.append({"double": float(s.rstrip("dD"))})
        elif re.fullmatch(r"-?\d+", s):
            vals.append({"int": int(s)})
        elif re.fullmatch(r"\(float\)\s*-?[\d.]+", s):
            vals.append({"float": float(s.split(")")[1])})
        elif re.fullmatch(r"\(long\)\s*-?\d+", s):
            vals.append({"long": int(s.split(")")[1])})
        else:
            raise ValueError("literal %r" % s)
    return vals


def strip_comments(body):
    out, i, n = [], 0, len(body)
    while i < n:
        c = body[i]
        if c == '"':
            j = i + 1
            while body[j] != '"':
                j += 2 if body[j] == "\\" else 1
            out.append(body[i:j + 1])
            i = j + 1
        elif body.startswith("//", i):
            while i < n and body[i] != "\n":
                i += 1
        elif body.startswith("/*", i):
            j = body.find("*/", i + 2)
            i = n if j < 0 else j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


# ---- query-API tests (FilterTestCase1/2): the Java builder calls restated as SiddhiQL
_JTOK = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?[fFdDlL]?)|'
                   r'(?P<id>[A-Za-z_]\w*)|(?P<p>[().,]))')


def _jtokens(text):
    out, i = [], 0
    while i < len(text):
        m = _JTOK.match(text, i)
        if not m or m.end() == i:
            if text[i:].strip() == "":
                break
            raise ValueError("java token at %r" % text[i:i + 20])
        i = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


def _jparse(toks, i=0):
    """primary ('.' name ['(' args ')'])* -> nested ('call', path, args) / ('str'|'num'|'id', v)."""
    kind, v = toks[i]
    i += 1
    if kind == "str":
        node = ("str", java_str(v))
    elif kind == "num":
        node = ("num", v)
    elif kind == "id":
        path = [v]
        while i + 1 < len(toks) and toks[i] == ("p", ".") and toks[i + 1][0] == "id":
            if i + 2 < len(toks) and toks[i + 2] == ("p", "("):
                break
            path.append(toks[i + 1][1])
            i += 2
        if i < len(toks) and toks[i] == ("p", ".") and i + 2 < len(toks) and toks[i + 2] == ("p", "("):
            path.append(toks[i + 1][1])
            i += 2
        if i < len(toks) and toks[i] == ("p", "("):
            args, i = _jargs(toks, i)
            node = ("call", ".".join(path), args)
        else:
            node = ("id", ".".join(path))
    else:
        raise ValueError("java expr at %r" % (v,))
    while i + 2 < len(toks) and toks[i] == ("p", ".") and toks[i + 1][0] == "id" and toks[i + 2] == ("p", "("):
        name = toks[i + 1][1]
        args, i = _jargs(toks, i + 2)
        node = ("meth", node, name, args)
    return node, i


def _jargs(toks, i):
    assert toks[i] == ("p", "(")
    i += 1
    args = []
    if toks[i] == ("p", ")"):
        return args, i + 1
    while True:
        a, i = _jparse(toks, i)
        args.append(a)
        if toks[i] == ("p", ")"):
            return args, i + 1
        if toks[i] != ("p", ","):
            raise ValueError("java args")
        i += 1


_CMP = {"EQUAL": "==", "NOT_EQUAL": "!=", "GREATER_THAN": ">", "GREATER_THAN_EQUAL": ">=",
        "LESS_THAN": "<", "LESS_THAN_EQUAL": "<="}
_MATH = {"add": "+", "subtract": "-", "multiply": "*", "divide": "/", "mod": "%"}


def _jexpr(n):
    """io.siddhi.query.api.expression.Expression builders -> SiddhiQL text."""
    if n[0] == "call":
        f, a = n[1].split(".")[-1], n[2]
        if f == "variable":
            return a[0][1]
        if f == "value":
            k, v = a[0]
            if k == "str":
                return "'%s'" % v
            if k == "id" and v in ("true", "false"):
                return v
            return v
        if f == "compare":
            return "(%s %s %s)" % (_jexpr(a[0]), _CMP[a[1][1].split(".")[-1]], _jexpr(a[2]))
        if f in _MATH:
            return "(%s %s %s)" % (_jexpr(a[0]), _MATH[f], _jexpr(a[1]))
        if f in ("and", "or"):
            return "(%s %s %s)" % (_jexpr(a[0]), f, _jexpr(a[1]))
        if f == "not":
            return "(not %s)" % _jexpr(a[0])
        if f == "isNull":
            return "(%s is null)" % _jexpr(a[0])
    raise ValueError("query-API expression %r" % (n,))


def _chain(n):
    """Flatten a builder chain: root call + [(method, args)]."""
    calls = []
    while n[0] == "meth":
        calls.append((n[2], n[3]))
        n = n[1]
    return n, calls[::-1]


def query_api_app(body):
    """SiddhiQL text of a test that builds its app with the query API
    (StreamDefinition.id(..).attribute(..), new Query().from/select/insertInto)."""
    types = {"STRING": "string", "INT": "int", "LONG": "long", "FLOAT": "float", "DOUBLE": "double", "BOOL": "bool"}
    defs = {}
    for m in re.finditer(r"StreamDefinition (\w+)\s*=\s*(StreamDefinition\.id\(.*?\));", body, re.S):
        root, calls = _chain(_jparse(_jtokens(m.group(2)))[0])
        attrs = ["%s %s" % (a[0][1], types[a[1][1].split(".")[-1]]) for name, a in calls if name == "attribute"]
        defs[m.group(1)] = "define stream %s (%s);" % (root[2][0][1], ", ".join(attrs))
    order = re.findall(r"siddhiApp\.defineStream\((\w+)\)", body)
    text = " ".join(defs[d] for d in order) + " "
    nq = len(re.findall(r"siddhiApp\.addQuery\(", body))
    if nq != 1:
        raise ValueError("query-API app with %d queries" % nq)
    ann = re.search(r'query\.annotation\(Annotation\.annotation\("info"\)\.element\("name",\s*"(\w+)"\)\);', body)
    fm = re.search(r"query\.from\((.*?)\);\s*query\.", body, re.S)
    sm = re.search(r"query\.select\((.*?)\);\s*query\.", body, re.S)
    im = re.search(r'query\.insertInto\("(\w+)"\);', body)
    if not (fm and sm and im):
        raise ValueError("query-API shape")
    root, calls = _chain(_jparse(_jtokens(fm.group(1)))[0])
    src = root[2][0][1]
    for name, a in calls:
        if name != "filter":
            raise ValueError("query-API input %s" % name)
        src += "[%s]" % _jexpr(a[0])
    root, calls = _chain(_jparse(_jtokens(sm.group(1)))[0])
    outs = []
    for name, a in calls:
        if name != "select":
            raise ValueError("query-API selector %s" % name)
        outs.append("%s as %s" % (_jexpr(a[1]), a[0][1]))
    q = "%sfrom %s select %s insert into %s;" % ("@info(name='%s') " % ann.group(1) if ann else "", src,
                                                 ", ".join(outs), im.group(1))
    return text + q


def _callback_bodies(body):
    """(name, QueryCallback|StreamCallback, body text) of each anonymous callback."""
    out = []
    for m in re.finditer(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)\(\)\s*\{', body):
        depth, i = 1, m.end()
        while depth and i < len(body):
            depth += {"{": 1, "}": -1}.get(body[i], 0)
            i += 1
        out.append((m.group(1), m.group(2), body[m.start():i]))
    return out


def _count_mult(cbody):
    """Events counted per in-event by a callback body (count.addAndGet(inEvents.length) k times)."""
    return (len(re.findall(r"count\.addAndGet\(inEvents\.length\)", cbody)) +
            len(re.findall(r"count\s*=\s*count\s*\+\s*inEvents\.length", cbody)) +
            len(re.findall(r"\bcount\s*\+=\s*inEvents\.length", cbody)))


def extract(name, body, line, fname):
    body = strip_comments(body)
    if re.search(r"executorService|Thread\(|persist\(|restore|setExtension", body):
        return None, "threads/persist/other"
    strings = {}
    # int constants spliced into app strings (`final int length = 4;` ... "length(" + length + ")")
    for m in re.finditer(r"(?:final\s+)?int (\w+)\s*=\s*(\d+)\s*;", body):
        strings[m.group(1)] = m.group(2)
    for m in re.finditer(r"String (\w+)\s*=\s*((?:\s*(?:" + STR_LIT + r"|\w+)\s*\+?)+)\s*;", body):
        try:
            strings[m.group(1)] = eval_concat(m.group(2), strings)
        except ValueError:
            pass
    m = re.search(r"createSiddhiAppRuntime\(([^;]*)\);", body)
    if not m:
        return None, "no app"
    try:
        if m.group(1).strip() == "siddhiApp" and "new SiddhiApp(" in body:
            app = query_api_app(body)
        else:
            app = eval_concat(m.group(1).replace("(", " ").replace(")", " "), strings)
    except (ValueError, KeyError, IndexError, AssertionError) as e:
        return None, "app: %s" % e
    cbs = re.findall(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)', body)
    # TestUtil.addQueryCallback(runtime, "q", new Object[]{..}, ...) (T/TestUtil.java:45-66):
    # expected rows in arrival order, counts read back through the TestCallback
    tu = list(re.finditer(r'TestUtil\.add(Query|Stream)Callback\(\s*\w+\s*,\s*"(\w+)"\s*(,(?:[^;])*?)?\)\s*;', body))
    tu_expected = []
    if tu:
        if cbs or len(tu) != 1:
            return None, "callbacks=%d" % (len(cbs) + len(tu))
        cb_kind = "QueryCallback" if tu[0].group(1) == "Query" else "StreamCallback"
        cb_name = tu[0].group(2)
        for k, em in enumerate(re.finditer(r"new\s+Object\[\]\s*\{(.*?)\}", tu[0].group(3) or "", re.S)):
            try:
                # TestQueryCallback checks expected[i] only for events that arrive
                tu_expected.append({"n": k + 1, "data": parse_values(em.group(1)), "if_arrived": True})
            except ValueError as e:
                return None, str(e)
    elif len(cbs) != 1:
        # several callbacks: the one that counts (FilterTestCase1: query1 counts, query2 only asserts)
        counting = [c for c in _callback_bodies(body) if _count_mult(c[2])]
        if len(counting) != 1:
            return None, "callbacks=%d" % len(cbs)
        cb_name, cb_kind = counting[0][0], counting[0][1]
    else:
        cb_name, cb_kind = cbs[0]
    playback = "@app:playback" in app.replace(" ", "").lower()
    handlers = dict(re.findall(r'InputHandler (\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body))
    # statement stream: sends, sleeps, clock updates
    clock = T0
    sends = []
    now_var = None
    events_ok = True
    stmt_re = re.compile(
        r"(?P<wait>TestUtil\.waitForInEvents\((?P<wms>\d+),\s*\w+,\s*(?P<wn>\d+)\))"
        r"|(?P<swait>SiddhiTestHelper\.waitForEvents\((?P<sms>\d+),\s*(?P<sn>\d+),\s*\w+(?:\.get\(\))?,\s*"
        r"(?P<sto>\d+)\))"
        r"|(?P<sleep>Thread\.sleep\((?P<ms>\d+)\))"
        r"|(?P<nowdecl>long (?P<nv>\w+) = (?P<nval>System\.currentTimeMillis\(\)|\d+L?);)"
        r"|(?P<nowadd>(?P<nv2>\w+) \+= (?P<addexpr>[\d *]+);)"
        r"|(?P<send>(?P<h>\w+)\.send\((?P<args>(?:[^;]|\n)*?)\);)")
    if tu:
        scan = body[tu[0].end():]
        # the expectations are read at the first assertion: later sleeps (after
        # shutdown) must not fire more timers
        cut = [i for i in (scan.find("AssertJUnit."), scan.find("throwAssertionErrors"), scan.find(".shutdown()"))
               if i >= 0]
        if cut:
            scan = scan[:min(cut)]
    else:
        cb_start = body.find("addCallback")
        cb_end = body.find("});", cb_start)
        scan = body[cb_end:] if cb_start >= 0 else body
        # wall-clock sleeps fire due timers up to the first count assertion
        cut = [i for i in (scan.find("AssertJUnit.assert"), scan.find(".shutdown()")) if i >= 0]
        if cut:
            scan = scan[:min(cut)]
    if re.search(r"\bfor\s*\(|\bwhile\s*\(|new Event\[|\.send\(new Event", scan):
        return None, "loop in sends"
    last_ts = None
    nv_value = None
    for sm in stmt_re.finditer(scan):
        if sm.group("wait"):
            # TestUtil.waitForInEvents (T/TestUtil.java:69-79): sleep, up to n times,
            # until exactly one event arrived; wall-clock timers fire meanwhile
            if not playback:
                sends.append({"wait": int(sm.group("wms")), "retry": int(sm.group("wn"))})
            clock += int(sm.group("wms"))
        elif sm.group("swait"):
            # SiddhiTestHelper.waitForEvents(sleep, n, counter, timeout)
            # (C/util/SiddhiTestHelper.java:49-57): sleep until the counter
            # reaches n or the timeout passed; wall-clock timers fire meanwhile
            if not playback:
                ms_ = int(sm.group("sms"))
                sends.append({"wait": ms_, "retry": int(sm.group("sto")) // ms_ + 1, "until": int(sm.group("sn"))})
            clock += int(sm.group("sms"))
        elif sm.group("sleep"):
            clock += int(sm.group("ms"))
            if playback and "idle.time" in app:
                # playback heartbeat: idle wall-clock time moves the app time
                sends.append({"idle": int(sm.group("ms"))})
            elif not playback:
                # wall clock: the scheduler fires due timers during the sleep
                sends.append({"time": clock})
        elif sm.group("nowdecl"):
            now_var = sm.group("nv")
            v = sm.group("nval")
            nv_value = clock if v.startswith("System") else int(v.rstrip("L"))
        elif sm.group("nowadd"):
            if sm.group("nv2") == now_var:
                nv_value += eval(sm.group("addexpr"))
        elif sm.group("send"):
            h = sm.group("h")
            if h not in handlers:
                return None, "unknown handler %s" % h
            args = sm.group("args").strip()
            am = re.fullmatch(r"(?:(?P<ts>[^,]+?)\s*,\s*)?new Object\[\]\s*\{(?P<vals>.*)\}", args, re.S)
            if not am:
                return None, "send form %r" % args[:40]
            try:
                # a wall-clock reading as an attribute value: the send's clock
                vals = parse_values(am.group("vals").replace("System.currentTimeMillis()", "%dL" % clock))
            except ValueError as e:
                return None, str(e)
            ts_expr = am.group("ts")
            if ts_expr is None:
                ts = clock
                clock += 1
            else:
                ts_expr = ts_expr.strip()
                if now_var and re.fullmatch(r"\+\+" + now_var, ts_expr):
                    nv_value += 1
                    ts = nv_value
                elif now_var and re.fullmatch(now_var + r"\s*\+\s*\d+", ts_expr):
                    ts = nv_value + int(ts_expr.split("+")[1])
                elif now_var and ts_expr == now_var:
                    ts = nv_value
                elif re.fullmatch(r"\d+L?", ts_expr):
                    ts = int(ts_expr.rstrip("L"))
                else:
                    return None, "ts expr %r" % ts_expr
            sends.append({"stream": handlers[h], "ts": ts, "data": vals})
    if not sends:
        return None, "no sends"
    # expectations
    cbm = re.search(r"addCallback\(.*?\}\s*\);", body, re.S)
    cbody = cbm.group(0) if cbm and not tu else ""
    if not tu:
        for name_, kind_, b_ in _callback_bodies(body):
            if name_ == cb_name:
                cbody = b_
    expected = list(tu_expected)
    cells = []
    # per-callback cell checks: "X".equals(inEvents[0].getData(k)) / assertEquals("X", inEvents[0].getData(k).toString())
    def _conditional(at):
        # inside `if (<condition on the event>) { ... }`: not a check of every chunk
        pre = cbody[:at].rstrip()
        if pre.endswith("AssertJUnit."):
            pre = pre[:-len("AssertJUnit.")].rstrip()
        k = pre.rfind("if (")
        return pre.endswith("{") and k >= 0 and ";" not in pre[k:]

    for cm_ in re.finditer(r'assertTrue\("([^"]*)"\.equals\(inEvents\[0\]\.getData\((\d+)\)\)\)', cbody):
        if not _conditional(cm_.start()):
            cells.append({"which": "first_of_each", "col": int(cm_.group(2)), "value": cm_.group(1)})
    for cm_ in re.finditer(r'assertEquals\("([^"]*)",\s*inEvents\[0\]\.getData\((\d+)\)\.toString\(\)\)', cbody):
        if not _conditional(cm_.start()):
            cells.append({"which": "first_of_each", "col": int(cm_.group(2)), "value": cm_.group(1)})
    cases = re.split(r"case (\d+):", cbody)
    if len(cases) > 1:
        for k in range(1, len(cases), 2):
            em = re.search(r"assertArrayEquals\(new Object\[\]\s*\{(.*?)\}\s*,", cases[k + 1], re.S)
            if em:
                try:
                    expected.append({"n": int(cases[k]), "data": parse_values(em.group(1))})
                except ValueError as e:
                    return None, str(e)
    else:
        ems = re.findall(r"assertArrayEquals\(new Object\[\]\s*\{(.*?)\}\s*,\s*(\w+)(\[0\])?\.getData\(\)", cbody, re.S)
        if len(ems) == 1:
            try:
                expected.append({"n": "all" if ems[0][2] == "" else "first_of_each", "data": parse_values(ems[0][0])})
            except ValueError as e:
                return None, str(e)
    # StreamCallback bodies that count events and check the n-th one:
    # `if (xCount == N) { assertEquals(V, event.getData()[K]); }` (a StreamCallback
    # sees every event as CURRENT: InsertIntoStreamCallback.send :50-57)
    nth = []
    if cb_kind == "StreamCallback" and not tu:
        if re.search(r"getData\(\)\[\d+\]\.equals\(", cbody):
            return None, "data-dependent callback counters"
        for cm_ in re.finditer(r"if \((\w+) == (\d+)\) \{\s*(?:AssertJUnit\.)?assertEquals\(([^,]+?),\s*"
                               r"event\.getData\(\)\[(\d+)\]\);", cbody):
            if not re.search(re.escape(cm_.group(1)) + r"\+\+", cbody):
                continue
            try:
                nth.append({"n": int(cm_.group(2)), "col": int(cm_.group(4)),
                            "value": parse_values(cm_.group(3))[0]})
            except ValueError as e:
                return None, str(e)
    count = None
    sizes = {}
    if tu:
        # the first count assertion after the callback (later ones follow more sends)
        cm = re.search(r'assertEquals\("[^"]*",\s*(\d+),\s*\w+\.getInEventCount\(\)\)', body[tu[0].end():])
        if cm:
            count = int(cm.group(1))
    for pat in [] if tu else [r'assertEquals\("Number of success events",\s*(\d+),\s*\w+\.getInEventCount\(\)\)',
                r'assertEquals\("Number of success events",\s*(\d+),\s*inEventCount\)',
                r"assertEquals\(inEventCount,\s*(\d+)\)",
                r'assertEquals\("[^"]*[Ee]vent count[^"]*",\s*(\d+),\s*inEventCount\)',
                r"assertEquals\((\d+),\s*inEventCount\)",
                r'assertEquals\("[^"]*",\s*(\d+),\s*inEventCount\)']:
        cm = re.search(pat, body)
        if cm:
            count = int(cm.group(1))
            break
    mult = _count_mult(cbody) if not tu else 0
    if count is None and mult:
        # `count.addAndGet(inEvents.length)` (k times per callback) checked with
        # assertEquals(N, count[.get()]) or, lacking an assertion, the count the
        # test waits for (SiddhiTestHelper.waitForEvents(sleep, N, count, timeout))
        after = body[body.find(cbody) + len(cbody):] if cbody else body
        cm = (re.search(r"assertEquals\((?:\"[^\"]*\",\s*)?(\d+)L?,\s*count(?:\.get\(\))?\)", after) or
              re.search(r"SiddhiTestHelper\.waitForEvents\(\d+,\s*(\d+),\s*count,", after))
        if cm:
            n_ = int(cm.group(1))
            if n_ % mult:
                return None, "count %d not a multiple of %d" % (n_, mult)
            count = n_ // mult
    removes = None
    for pat in [r'assertEquals\("Number of remove events",\s*(\d+),\s*(?:removeEventCount|\w+\.getRemoveEventCount\(\))\)',
                r'assertEquals\("[^"]*[Rr]emove event count[^"]*",\s*(\d+),\s*removeEventCount\)',
                r"assertEquals\((\d+),\s*removeEventCount\)"]:
        rm = re.search(pat, body)
        if rm:
            removes = int(rm.group(1))
            break
    if cb_kind == "StreamCallback" and re.search(r"\bevents\.length == \d+\)", cbody):
        # counters bumped per callback by chunk size: the checkable number is the
        # total the callback saw (`for (Event event : events) count++`)
        tm = re.search(r'assertEquals\("Total events",\s*(\d+),\s*count\)', body)
        if not tm or not re.search(r"for \(Event \w+ : events\)", cbody) or "count++" not in cbody:
            return None, "per-chunk-size counters"
        count, removes = int(tm.group(1)), None
        # `if (events.length == k) { c++; }` checked by assertEquals(..., n, c):
        # n callback chunks of k events
        for km in re.finditer(r"events\.length == (\d+)\)\s*\{\s*(\w+)\+\+;", cbody):
            am = re.search(r'assertEquals\((?:"[^"]*",\s*)?(\d+),\s*' + km.group(2) + r"\)", body)
            if am:
                sizes[int(km.group(1))] = int(am.group(1))
    if cb_kind == "StreamCallback" and count is None and removes is not None and "inEventCount++" not in cbody:
        # a StreamCallback counter named removeEventCount counts every event it sees
        count, removes = removes, None
    if count is None and not expected and not cells and not nth:
        return None, "no expectations"
    return {
        "name": "%s.%s" % (os.path.basename(fname)[:-5], name),
        "source": "modules/siddhi-core/src/test/java/io/siddhi/core/%s:%d" % (fname, line),
        "app": app,
        "callback": {"kind": "query" if cb_kind == "QueryCallback" else "stream", "name": cb_name},
        "sends": sends,
        "expected_rows": expected,
        "expected_count": count,
        "expected_remove_count": removes,
        "expected_chunk_sizes": {str(k): v for k, v in sorted(sizes.items())},
        "expected_cells": cells,
        "expected_nth": nth,
        "playback": "@app:playback" in app.replace(" ", "").lower() or "@app:playback" in app.lower(),
        "start_time": None if playback else T0,
    }, None


# Expectations a test states through callback-side counter logic rather than
# assertArrayEquals, transcribed by hand (the assertion they follow is cited):
# lengthWindowTest2 (query/window/LengthWindowTestCase.java:105-114) checks that
# with length 4 the StreamCallback sees events 1..4, then each later event
# preceded by the expired event it evicts (volumes 1, 5, 2, 6 in turn).
_F = lambda x: {"float": x}
_I = lambda x: {"int": x}
MANUAL_ROWS = {
    "LengthWindowTestCase.lengthWindowTest2": [
        {"n": i + 1, "data": d} for i, d in enumerate([
            ["IBM", _F(700.0), _I(1)], ["WSO2", _F(60.5), _I(2)], ["IBM", _F(700.0), _I(3)],
            ["WSO2", _F(60.5), _I(4)], ["IBM", _F(700.0), _I(1)], ["IBM", _F(700.0), _I(5)],
            ["WSO2", _F(60.5), _I(2)], ["WSO2", _F(60.5), _I(6)]])],
}


def main():
    os.makedirs(OUT, exist_ok=True)
    total, skipped = 0, {}
    for f in FILES:
        path = REF + f
        if not os.path.exists(path):
            print("missing", f)
            continue
        text = open(path).read()
        cases = []
        for name, body, line, ann in split_methods(text):
            if "expectedExceptions" in ann:
                continue
            case, why = extract(name, body, line, f)
            if case is None:
                skipped[f + ":" + name] = why
                continue
            if case["name"] in MANUAL_ROWS:
                case["expected_rows"] = MANUAL_ROWS[case["name"]]
            cases.append(case)
        total += len(cases)
        with open(os.path.join(OUT, os.path.basename(f)[:-5] + ".json"), "w") as fp:
            json.dump(cases, fp, indent=1)
        print("%-55s %3d cases" % (f, len(cases)))
    print("total", total, "skipped", len(skipped))
    if "-v" in sys.argv:
        for k, v in skipped.items():
            print("  skip", k, v)


if __name__ == "__main__":
    main()
