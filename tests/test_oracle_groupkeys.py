"""Group-by key identity on the CPU oracle (the checker the device group
dictionary is compared with): the reference's key is the text of the values
(C/query/selector/GroupByKeyGenerator.java:63-73), so a null string and the
string "null" share a group, every NaN is one group and 0.0 / -0.0 are two."""
from oracle_engine import OracleQueryEngine
from siddhi_amd import runtime as rt


def _run(app, stream, rows):
    mgr = rt.SiddhiManager(engine_factory=OracleQueryEngine)
    r = mgr.createSiddhiAppRuntime(app)
    got = []
    class QC(rt.QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend(e.getData() for e in (ins or []))
    r.addCallback("q", QC())
    r.start()
    h = r.getInputHandler(stream)
    for i, row in enumerate(rows):
        h.send(1000 + i, row)
    r.shutdown()
    return got


def test_null_string_is_the_string_null():
    app = ("@app:playback define stream S (s string, v double); "
           "@info(name='q') from S#window.length(10) select s, count() as c group by s insert into O;")
    got = _run(app, "S", [["null", 1.0], [None, 2.0], ["x", 3.0], [None, 4.0]])
    assert [g[1] for g in got] == [1, 2, 1, 3]


def test_nan_one_group_signed_zeros_two():
    app = ("@app:playback define stream S (k double, v double); "
           "@info(name='q') from S#window.length(10) select k, count() as c group by k insert into O;")
    nan = float("nan")
    got = _run(app, "S", [[nan, 1.0], [nan, 1.0], [0.0, 1.0], [-0.0, 1.0], [0.0, 1.0]])
    assert [g[1] for g in got] == [1, 2, 1, 1, 2]


def test_multi_attribute_and_null_int_key():
    app = ("@app:playback define stream S (s string, i int, v double); "
           "@info(name='q') from S#window.length(10) select s, i, count() as c group by s, i insert into O;")
    got = _run(app, "S", [["a", None, 1.0], ["a", 1, 1.0], ["a", None, 1.0], ["b", None, 1.0]])
    assert [g[2] for g in got] == [1, 1, 2, 1]
