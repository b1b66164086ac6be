"""Fast-path filter predicates (dev_expr.h eval_fpred) against the bytecode
interpreter and the CPU oracle: a matrix of comparison / arithmetic shapes over
int, long, float and double columns with nulls, division by zero (null) and
mixed-type promotion.  SHD_NO_FAST_PRED=1 forces the interpreter."""
import numpy as np
import pytest

from parity import assert_same_rows, compile_single_query, run_device, run_oracle
from siddhi_amd.runtime import ColumnBatch

pytestmark = pytest.mark.gpu

DEF = "define stream S (i int, l long, f float, d double, s string);"
FILTERS = [
    "i > 10", "l <= 20", "f < 30.5", "d >= 40", "i == l", "f != d", "i * 2 > l", "d / i > 3.0",
    "l % i == 1", "f * 1.5 <= d", "i + l > d and f < 50", "d - f > 0 and i != 7 and l > 3",
    "i / 0 > 1", "s == 'k3'", "d > l * 1.05",
]


def batch(n, seed):
    rng = np.random.default_rng(seed)
    i = rng.integers(-5, 60, n).astype(np.int32)
    l = rng.integers(-5, 60, n).astype(np.int64)
    f = (rng.random(n) * 60).astype(np.float32)
    d = rng.random(n) * 60
    s = rng.integers(0, 6, n).astype(np.uint32)
    nulls = [(rng.random(n) < 0.1).astype(np.uint8) for _ in range(5)]
    ts = 1000 + np.arange(n, dtype=np.int64)
    return ColumnBatch(ts, [i, l, f, d, s], nulls, np.array([0, n], np.int64))


@pytest.mark.parametrize("flt", FILTERS)
def test_fast_predicate_equals_interpreter_and_oracle(hip_available, monkeypatch, flt):
    app = "@app:playback " + DEF + " @info(name='q') from S[" + flt + "] select i, l, f, d insert into O;"
    from siddhi_amd import planner as pl
    d = pl.StringDictionary()
    for k in range(6):
        d.id("k%d" % k)
    qp, _ = compile_single_query(app, d)
    b = batch(5000, hash(flt) % 1000)
    batches = [(0, b)]
    ora = run_oracle(qp, batches)
    fast = run_device(qp, batches)[0]
    monkeypatch.setenv("SHD_NO_FAST_PRED", "1")
    slow = run_device(qp, batches)[0]
    assert_same_rows(fast, ora)
    assert_same_rows(slow, ora)
