"""`output snapshot every <time>` on non-windowed queries (PerSnapshot /
GroupByPerSnapshotOutputRateLimiter, C/query/output/ratelimit/snapshot/).

The reference's own tests (T/query/ratelimit/SnapshotOutputRateLimitTestCase
.java testSnapshotOutputRateLimitQuery1-4) run on the wall clock with
Thread.sleep between sends; tests/golden/make_kats.py cannot extract them (no
literal expectations).  They are restated here on a fixed clock: the app
starts at wall time 0 (scheduledTime = 0 + 1000), each send carries the time
it was made, each sleep is an advanceTime to the time it ends, and the
asserted counts / values are the Java test's.  Parity pinned by those
assertions only (bundle and event counts, the values they allow).
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle_engine import OracleQueryEngine  # noqa: E402
from siddhi_amd import planner as pl  # noqa: E402
from siddhi_amd.runtime import SiddhiManager, StreamCallback  # noqa: E402

DEF = "define stream LoginEvents (timestamp long, ip string);"
Q_PLAIN = ("@info(name = 'query1') from LoginEvents select ip "
           "output snapshot every 1 sec insert all events into uniqueIps ;")
Q_GROUP = ("@info(name = 'query1') from LoginEvents select ip group by ip "
           "output snapshot every 1 sec insert all events into uniqueIps ;")


def _run(app, script, device=False):
    """script: ("send", t, ip) | ("sleep_to", t); returns the callback bundles."""
    m = SiddhiManager() if device else SiddhiManager(engine_factory=OracleQueryEngine)
    rt = m.createSiddhiAppRuntime(app)
    now = [0]
    rt.clock = lambda: now[0]
    bundles = []

    class CB(StreamCallback):
        def receive(self, events):
            bundles.append([(e.data[0], e.is_expired) for e in events])

    rt.addCallback("uniqueIps", CB())
    rt.start()
    ih = rt.getInputHandler("LoginEvents")
    for step in script:
        if step[0] == "send":
            now[0] = step[1]
            ih.send(step[1], [step[1], step[2]])
        else:
            now[0] = step[1]
            rt.advanceTime(step[1])
    rt.shutdown()
    return bundles


# testSnapshotOutputRateLimitQuery1: send .5, sleep 10, send .3, wait for one event
SCRIPT1 = [("send", 0, "192.10.1.5"), ("send", 10, "192.10.1.3"), ("sleep_to", 1000)]
# Query2: sleep 1200, send .5, sleep 500, send .3, sleep 2200
SCRIPT2 = [("sleep_to", 1200), ("send", 1200, "192.10.1.5"), ("sleep_to", 1700), ("send", 1700, "192.10.1.3"),
           ("sleep_to", 3900)]
# Query3: send .5, sleep 100, send .3, sleep 2200, send .9, sleep 100, send .4, sleep 1100
SCRIPT3 = [("send", 0, "192.10.1.5"), ("sleep_to", 100), ("send", 100, "192.10.1.3"), ("sleep_to", 2300),
           ("send", 2300, "192.10.1.9"), ("sleep_to", 2400), ("send", 2400, "192.10.1.4"), ("sleep_to", 3500)]
# Query4 (group by ip): sleep 1100, send .5, .3, sleep 2200, send .5, .4, sleep 1200
SCRIPT4 = [("sleep_to", 1100), ("send", 1100, "192.10.1.5"), ("send", 1100, "192.10.1.3"), ("sleep_to", 3300),
           ("send", 3300, "192.10.1.5"), ("send", 3300, "192.10.1.4"), ("sleep_to", 4500)]


def _check_plain(bundles, n, allowed):
    evs = [e for b in bundles for e in b]
    assert not any(x for _, x in evs), "Remove events emitted"
    assert len(evs) == n
    assert all(ip in allowed for ip, _ in evs)


def _cases(device):
    b = _run(DEF + Q_PLAIN, SCRIPT1, device)
    _check_plain(b, 1, {"192.10.1.3"})
    b = _run(DEF + Q_PLAIN, SCRIPT2, device)
    _check_plain(b, 2, {"192.10.1.3"})
    b = _run(DEF + Q_PLAIN, SCRIPT3, device)
    _check_plain(b, 3, {"192.10.1.3", "192.10.1.4"})
    b = _run(DEF + Q_GROUP, SCRIPT4, device)
    assert len(b) == 3 and sum(len(x) for x in b) == 7
    # what the LinkedHashMap holds at each TIMER (2000, 3000, 4000), in first-arrival order
    assert [[ip for ip, _ in x] for x in b] == [["192.10.1.5", "192.10.1.3"]] * 2 + \
        [["192.10.1.5", "192.10.1.3", "192.10.1.4"]]


def test_snapshot_limiters_oracle():
    _cases(False)


@pytest.mark.gpu
def test_snapshot_limiters_device(hip_available):
    _cases(True)


def test_snapshot_flush_on_event_time():
    # an event at or past scheduledTime flushes what was held before it is held
    # itself (tryFlushEvents before state.lastEvent = event)
    b = _run(DEF + Q_PLAIN, [("send", 100, "a"), ("send", 1000, "b"), ("send", 1500, "c"), ("sleep_to", 2000)])
    assert [[ip for ip, _ in x] for x in b] == [["a"], ["c"]]


@pytest.mark.parametrize("q", [
    "from LoginEvents#window.length(2) select ip output snapshot every 1 sec insert into O;",
    "from LoginEvents select ip, count() as c output snapshot every 1 sec insert into O;",
])
def test_snapshot_refused_where_inexact(q):
    m = SiddhiManager(engine_factory=OracleQueryEngine)
    with pytest.raises(pl.UnsupportedPlanException):
        m.createSiddhiAppRuntime(DEF + q)
