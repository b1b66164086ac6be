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
    "query/window/LengthWindowTestCase.java",
    "query/window/TimeWindowTestCase.java",
    "query/GroupByTestCase.java",
    "query/FilterTestCase1.java",
    "query/FilterTestCase2.java",
    "query/pattern/absent/AbsentPatternTestCase.java",
    "query/pattern/absent/AbsentWithEveryPatternTestCase.java",
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


def extract(name, body, line, fname):
    body = strip_comments(body)
    if re.search(r"executorService|Thread\(|persist\(|restore|setExtension", body):
        return None, "threads/persist/other"
    strings = {}
    for m in re.finditer(r"String (\w+)\s*=\s*((?:\s*" + STR_LIT + r"\s*\+?)+)\s*;", body):
        strings[m.group(1)] = eval_concat(m.group(2), strings)
    m = re.search(r"createSiddhiAppRuntime\(([^;]*)\);", body)
    if not m:
        return None, "no app"
    try:
        app = eval_concat(m.group(1).replace("(", " ").replace(")", " "), strings)
    except ValueError as e:
        return None, str(e)
    cbs = re.findall(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)', body)
    if len(cbs) != 1:
        return None, "callbacks=%d" % len(cbs)
    cb_name, cb_kind = cbs[0]
    handlers = dict(re.findall(r'InputHandler (\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body))
    # statement stream: sends, sleeps, clock updates
    clock = T0
    sends = []
    now_var = None
    events_ok = True
    stmt_re = re.compile(
        r"(?P<sleep>Thread\.sleep\((?P<ms>\d+)\))"
        r"|(?P<nowdecl>long (?P<nv>\w+) = (?P<nval>System\.currentTimeMillis\(\)|\d+L?);)"
        r"|(?P<nowadd>(?P<nv2>\w+) \+= (?P<addexpr>[\d *]+);)"
        r"|(?P<send>(?P<h>\w+)\.send\((?P<args>(?:[^;]|\n)*?)\);)")
    cb_start = body.find("addCallback")
    cb_end = body.find("});", cb_start)
    scan = body[cb_end:] if cb_start >= 0 else body
    if re.search(r"\bfor\s*\(|\bwhile\s*\(|new Event\[|\.send\(new Event", scan):
        return None, "loop in sends"
    last_ts = None
    nv_value = None
    for sm in stmt_re.finditer(scan):
        if sm.group("sleep"):
            clock += int(sm.group("ms"))
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
                vals = parse_values(am.group("vals"))
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
    cbody = cbm.group(0) if cbm else ""
    expected = []
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
    count = None
    for pat in [r'assertEquals\("Number of success events",\s*(\d+),\s*inEventCount\)',
                r"assertEquals\(inEventCount,\s*(\d+)\)",
                r'assertEquals\("[^"]*[Ee]vent count[^"]*",\s*(\d+),\s*inEventCount\)',
                r"assertEquals\((\d+),\s*inEventCount\)",
                r'assertEquals\("[^"]*",\s*(\d+),\s*inEventCount\)']:
        cm = re.search(pat, body)
        if cm:
            count = int(cm.group(1))
            break
    removes = None
    rm = re.search(r'assertEquals\("Number of remove events",\s*(\d+),\s*removeEventCount\)', body)
    if rm:
        removes = int(rm.group(1))
    if count is None and not expected:
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
        "playback": "@app:playback" in app.replace(" ", "").lower() or "@app:playback" in app.lower(),
    }, None


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
