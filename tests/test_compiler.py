"""SiddhiQL subset compiler + planner (host side, CPU)."""
import struct

import pytest

from siddhi_amd import planner as pl
from siddhi_amd import query_compiler as qc
from siddhi_amd import workloads as wl


def plan_of(app_text, qi=0):
    app = qc.parse(app_text)
    item = app.execution_order[qi]
    d = pl.StringDictionary()
    if isinstance(item, qc.Partition):
        return pl.plan_query(app, item.queries[0], d, item)
    return pl.plan_query(app, item, d)


@pytest.mark.parametrize("name", list(wl.CONFIGS))
def test_configs_compile(name):
    qp = plan_of(wl.CONFIGS[name][0])
    words = struct.unpack("<%di" % (len(qp.ir) // 4), qp.ir)
    assert words[0] == pl.MAGIC and words[1] == pl.VERSION


def test_p1_shape_is_every_then_stream():
    qp = plan_of(wl.P1_APP)
    assert qp.plan.shape.get("every_a_then_b")
    assert qp.plan.within == 1000
    assert qp.output_types == [pl.T_STRING, pl.T_DOUBLE, pl.T_DOUBLE]
    assert qp.receiver_kind == {"StockStream": "multi"}


def test_logical_parses_element_two_first():
    # StateInputStreamParser.java:349-361 parses stream element 2 before element 1
    qp = plan_of("define stream A (x int); define stream B (x int); "
                 "from e1=A and e2=B select e1.x as a, e2.x as b insert into O;")
    assert [m.ref for m in qp.plan.states] == ["e2", "e1"]


def test_compare_promotion_rules():
    assert pl.compare_type(">", pl.T_FLOAT, pl.T_LONG) == pl.T_FLOAT
    assert pl.compare_type("==", pl.T_FLOAT, pl.T_LONG) == pl.T_DOUBLE
    assert pl.compare_type("==", pl.T_INT, pl.T_LONG) == pl.T_LONG
    assert pl.compare_type("<", pl.T_INT, pl.T_DOUBLE) == pl.T_DOUBLE


def test_last_index_inside_own_filter_stays_previous():
    # ExpressionParser.java:1378-1385: e2[last] inside e2's own filter = LAST (previous)
    qp = plan_of("define stream A (price double); "
                 "from every e1=A, e2=A[price>e2[last].price]<2:5> select e1.price as p insert into O;")
    loads = [ins for e in qp.plan.exprs for ins in e if ins[0] == pl.OP_LOAD and ins[1] == 1 and ins[2] != -1]
    assert any(ins[2] == pl.IDX_LAST for ins in loads)


def test_unsupported_reports_reason():
    with pytest.raises(pl.UnsupportedPlanException):
        plan_of("define stream A (x int); from A#window.frequent(2) select x insert into O;")
    with pytest.raises(pl.UnsupportedPlanException):   # timeBatch's nextEmitTime is per processor
        plan_of("define stream A (x int); partition with (x of A) begin "
                "from A#window.timeBatch(1 sec) select x insert into O; end;")


def test_time_units():
    app = qc.parse("define stream A (x int); from every e1=A -> e2=A within 1 min 30 sec select e1.x as a insert into O;")
    assert app.queries[0].input.within_ms == 90_000


def test_partition_inner_stream_rewrite():
    """`insert into #S` / `from #S` inside a partition: the producer's rows
    carry its instance's key as the hidden `__pkey`, read through the first
    keyed pattern state (or the single input stream), and #S joins the
    partition keyed by it (PatternPartitionTestCase 32/33 shapes)."""
    app = qc.parse(
        "define stream S1 (symbol string, price float, volume int, q int); "
        "define stream S2 (symbol string, price float, volume int, q int); "
        "partition with (q of S1, q of S2) begin "
        "from every e1 = S1 -> e2 = S2[price > e1.price] select e1.symbol as s, e2.price as p insert into #Mid; "
        "from #Mid[p > 1.0] select s, p insert into Out; "
        "from S1 select symbol, volume insert into #Raw; "
        "from #Raw select symbol insert into Out2; end;")
    p = app.partitions[0]
    keys = {sid: e for e, sid in p.with_}
    assert keys["#Mid"] == qc.Var("__pkey") and keys["#Raw"] == qc.Var("__pkey")
    prod, cons, prod2, cons2 = p.queries
    assert prod.target == "#Mid" and not prod.inner_target
    assert prod.selector.attrs[-1].name == "__pkey"
    assert prod.selector.attrs[-1].expr == qc.Var("q", "e1")
    assert prod2.selector.attrs[-1].expr == qc.Var("q")
    assert cons.input.stream == "#Mid" and cons2.input.stream == "#Raw"
    assert [o.name for o in cons.selector.attrs] == ["s", "p"]
