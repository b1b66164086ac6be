"""Host side of query sharing (planner.share_groups / plan_shared_leader) and
the property the device groups rest on, checked on the CPU oracle: for
`every e1=A[f1_g] -> e2=B[f2] within W`, query g's rows are exactly the
leader's (f1 = the members' disjunction) whose e1 passes f1_g, in the
leader's order (each partial meets the later events alone,
ST/StreamPreStateProcessor.java:118-129,326-403)."""
import numpy as np

from parity import run_oracle, stock_batch
from siddhi_amd import planner as pl
from siddhi_amd import query_compiler as qc
from siddhi_amd import workloads as wl


def test_m5_pattern_variants_form_one_group():
    app = qc.parse(wl.M5_APP)
    qs = list(app.execution_order)
    groups = pl.share_groups(qs)
    # the 50 P1 variants, and the 50 W2-length variants (window lengths 100..5000)
    assert groups == [list(range(50)), list(range(50, 100))]
    lf = pl.leader_e1_filters([pl._e1_site(qs[i]).filters for i in groups[0]])
    assert len(lf) == 1 and lf[0].op == ">" and lf[0].right.value == 60.0


def test_window_leader_holds_the_longest_window():
    app = qc.parse(wl.M5_APP)
    qs = list(app.execution_order)
    d = pl.StringDictionary()
    wl.register_symbols(d, 10)
    lead = pl.plan_shared_leader(app, qs[50:], d)
    assert lead.plan.handlers[-1][2] == 5000   # (kind, window kind, length, second parameter)
    # a different filter (or aggregate, or group-by) is another group
    other = qc.parse(wl.M5_APP.replace("from StockStream[price>60]#window.length(400)",
                                       "from StockStream[price>61]#window.length(400)"))
    assert pl.share_signature(list(other.execution_order)[53]) != pl.share_signature(qs[52])


def test_share_signature_separates_other_differences():
    base = ("@app:playback " + wl.STOCK_DEF + " from every e1=StockStream[price>%s] -> "
            "e2=StockStream[symbol==e1.symbol and price>e1.price*%s] within %s "
            "select e1.symbol as symbol, e1.price as p1 insert into O;")
    sig = lambda *a: pl.share_signature(qc.parse(base % a).execution_order[0])
    assert sig(70, 1.05, "1 sec") == sig(75, 1.05, "1 sec")
    assert sig(70, 1.05, "1 sec") != sig(70, 1.06, "1 sec")
    assert sig(70, 1.05, "1 sec") != sig(70, 1.05, "2 sec")
    # a sequence or a non-`every` start is not shareable
    seq = qc.parse("@app:playback " + wl.STOCK_DEF + " from every e1=StockStream, e2=StockStream[price>e1.price] "
                   "select e1.price as p insert into O;").execution_order[0]
    assert pl.share_signature(seq) is None


def test_leader_filters_mixed_shapes_take_the_disjunction():
    f = lambda s: qc.parse("@app:playback " + wl.STOCK_DEF + " from every e1=StockStream[%s] -> "
                           "e2=StockStream[price>e1.price] select e1.price as p insert into O;" % s
                           ).execution_order[0].input.element.a.inner.filters
    lf = pl.leader_e1_filters([f("price > 70"), f("volume < 5")])
    assert len(lf) == 1 and lf[0].op == "or"
    assert pl.leader_e1_filters([f("price < 70"), f("price < 75")])[0].right.value == 75
    assert pl.leader_e1_filters([f("price > 70"), f("price >= 75")])[0].op == "or"


def test_oracle_member_rows_are_leader_rows_filtered_by_member_f1():
    app = qc.parse(wl.m5_app(6, 0))
    qs = list(app.execution_order)
    d = pl.StringDictionary()
    wl.register_symbols(d, 200)
    leader = pl.plan_shared_leader(app, qs, d)
    sym, price, vol, ts = wl.stock_stream(20_000, 200, 0.05, seed_offset=9)
    batches = [(0, stock_batch(sym[:12_000], price[:12_000], vol[:12_000], ts[:12_000])),
               (0, stock_batch(sym[12_000:], price[12_000:], vol[12_000:], ts[12_000:]))]
    lead_rows = run_oracle(leader, batches)
    p1 = lead_rows[3][:, 1].view(np.float64)
    assert len(p1) > 0
    for th, q in zip(wl.M5_PATTERN_THRESHOLDS, qs):
        rows = run_oracle(pl.plan_query(app, q, d), batches)
        keep = p1 > th
        assert np.array_equal(rows[3], lead_rows[3][keep])
        assert np.array_equal(rows[2], lead_rows[2][keep])
