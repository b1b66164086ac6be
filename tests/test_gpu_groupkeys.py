"""Group-by keys the reference accepts on a sliding window, on the device
(engine_single.hip: dense ids for one string / bool attribute, the device
group dictionary GDict for every other key) against the CPU oracle.

The reference's group key is the text String.valueOf(v1) + ":-:" + ...
(C/query/selector/GroupByKeyGenerator.java:63-73), so:
  * a null key is a group of its own (the text "null") -- for a string
    attribute the same group as the string "null";
  * negative ints, longs beyond 2^26 / 2^32, floats and doubles are keys;
  * every NaN is one key, 0.0 and -0.0 are two;
  * several attributes form one key.
Every test pushes several micro-batches, so the dictionary is carried and
grown across pushes; doubles within 1e-9 relative (segmented scans), exact
mode bit-exact."""
import numpy as np
import pytest

from parity import assert_rows_agg, compile_single_query, run_device, run_oracle
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

SCHEMA = "define stream S (s string, i int, l long, f float, d double, b bool); "


def make_batches(seed, nbatch, m, call=250):
    rng = np.random.default_rng(seed)
    out = []
    t = 10_000
    for j in range(nbatch):
        s = rng.integers(0, 40, m).astype(np.uint32)          # dictionary ids
        i = rng.choice(np.array([-7, -1, 0, 3, 2 ** 31 - 1, -2 ** 31, 123456789], np.int32), m)
        lv = rng.choice(np.array([-5, 1 << 26, (1 << 26) + 1, 1 << 40, -(1 << 62), 7], np.int64), m)
        f = rng.choice(np.array([0.0, -0.0, 1.5, np.nan, -2.25, np.inf], np.float32), m)
        d = rng.uniform(0, 100, m)
        dk = rng.choice(np.array([0.0, -0.0, np.nan, 1e300, -3.5], np.float64), m)
        b = rng.integers(0, 2, m).astype(np.uint8)
        nl = [(rng.random(m) < 0.08).astype(np.uint8) for _ in range(6)]
        ts = t + np.sort(rng.integers(0, 3000, m)).astype(np.int64)
        t = int(ts[-1])
        offs = np.arange(0, m + 1, call, dtype=np.int64)
        if offs[-1] != m:
            offs = np.append(offs, m)
        # column 4 (d) carries the aggregated values; the double key is column 4 of a
        # second schema below, so keep both shapes in one generator
        out.append((ColumnBatch(ts, [s, i, lv, f, d, b], nl, offs), dk))
    return out


APPS = [
    ("int-neg-large", "from S#window.length(300) select i, sum(d) as sd, count() as c group by i insert into O;"),
    ("long-wide", "from S#window.time(40 milliseconds) select l, avg(d) as a, count() as c group by l insert into O;"),
    ("float-nan-zero", "from S#window.length(200) select f, sum(d) as sd, count() as c group by f insert into O;"),
    ("string-null", "from S#window.length(500) select s, avg(d) as a, count() as c group by s insert into O;"),
    ("bool-null", "from S#window.length(100) select b, sum(d) as sd, count() as c group by b insert into O;"),
    ("multi-attr", "from S[d > 5.0]#window.length(400) select s, i, sum(d) as sd, count() as c group by s, i "
                   "insert into O;"),
    ("multi-4", "from S#window.time(25 milliseconds) select s, l, f, b, count() as c, avg(d) as a "
                "group by s, l, f, b insert into O;"),
]


@pytest.mark.parametrize("exact", [False, True], ids=["scan", "exact"])
@pytest.mark.parametrize("name,app", APPS, ids=[a[0] for a in APPS])
def test_group_keys_equal_oracle(hip_available, name, app, exact):
    qp, d = compile_single_query("@app:playback " + SCHEMA + app)
    # make string id 11 the string "null" for the string-null case
    batches = [(0, b) for b, _ in make_batches(sum(name.encode()), 4, 6_000)]
    if name == "string-null":
        nid = d.id("null")
        for _, b in batches:
            b.cols[0][b.cols[0] == 11] = nid
    ora = run_oracle(qp, batches)
    dev, _, kind = run_device(qp, batches, exact=exact)
    assert kind == 2 and len(ora[2]) > 0
    assert_rows_agg(dev, ora, qp, exact=exact)


def test_double_keys_and_dictionary_growth(hip_available):
    """Double keys (NaN, +-0.0) and a dictionary that grows across pushes:
    every push brings keys never seen before."""
    app = ("@app:playback define stream D (k double, v double); "
           "from D#window.length(700) select k, sum(v) as s, count() as c group by k insert into O;")
    qp, _ = compile_single_query(app)
    rng = np.random.default_rng(5)
    batches = []
    t = 1000
    for j in range(5):
        m = 20_000
        k = rng.integers(0, 3000 * (j + 1), m).astype(np.float64) * 0.5 - 17.0
        k[rng.random(m) < 0.05] = np.nan
        k[rng.random(m) < 0.05] = -0.0
        v = rng.uniform(0, 10, m)
        nl = (rng.random(m) < 0.03).astype(np.uint8)
        ts = t + np.arange(m, dtype=np.int64)
        t = int(ts[-1]) + 1
        batches.append((0, ColumnBatch(ts, [k, v], [nl, None], np.arange(0, m + 1, 500, dtype=np.int64))))
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)


def test_forced_dictionary_for_string_keys(hip_available, monkeypatch):
    """SHD_GROUP_DICT=1 puts string keys on the dictionary path too (the W2
    shape): same rows as the dense ids."""
    monkeypatch.setenv("SHD_GROUP_DICT", "1")
    qp, _ = compile_single_query("@app:playback " + SCHEMA + APPS[3][1])
    batches = [(0, b) for b, _ in make_batches(3, 3, 8_000)]
    ora = run_oracle(qp, batches)
    dev, _, _ = run_device(qp, batches)
    assert_rows_agg(dev, ora, qp, exact=False)
