"""The CPU oracle against the reference's own end-to-end tests:
expectations transcribed by tests/golden/make_kats.py from
modules/siddhi-core/src/test/java/io/siddhi/core/**.  CPU only."""
import pytest

from kat_runner import check_case, load_cases, run_case
from oracle_engine import OracleQueryEngine
from siddhi_amd.planner import UnsupportedPlanException
from siddhi_amd.query_compiler import OutOfScopeSyntax

CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_kat(case):
    try:
        col = run_case(case, OracleQueryEngine)
    except (UnsupportedPlanException, OutOfScopeSyntax) as e:
        pytest.skip("outside the hot path: %s" % e)
    errs = check_case(case, col)
    assert not errs, "%s (%s): %s" % (case["name"], case["source"], errs)


def test_kat_corpus_size():
    # the corpus must keep covering the hot-path test files
    names = {c["name"].split(".")[0] for c in CASES}
    for f in ("EveryPatternTestCase", "CountPatternTestCase", "LogicalPatternTestCase", "WithinPatternTestCase",
              "SequenceTestCase", "PatternPartitionTestCase", "SequencePartitionTestCase", "PlaybackTestCase"):
        assert f in names
    assert len(CASES) >= 150
