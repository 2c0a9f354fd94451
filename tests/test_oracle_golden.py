"""Pins the CPU oracle (oracle/popbam_oracle.cpp) to the reference: for every golden case
the oracle's TSV must equal, byte for byte, what the compiled reference printed on the same
BAM (tests/golden/*/out, made by tests/golden/make_golden.py).  No GPU needed."""
import pytest

import fixtures
import harness

CASES = harness.all_cases()


@pytest.mark.parametrize("name,idx", CASES, ids=[f"{n}-{i:02d}" for n, i in CASES])
def test_oracle_matches_reference(name, idx):
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    assert cs["rc"] == 0
    st = harness.Setup(name, cs["args"], cs["region"])
    ours = harness.oracle_run(st)
    gold = fixtures.golden_text(name, cs["stdout"])
    ok, diff = harness.same_output(cs["args"], gold, ours)
    assert ok, f"{cs['args']} {cs['region']}\n gold: {diff[0]}\n ours: {diff[1]}"


def test_fixture_coverage():
    """The golden set exercises the quirks SURVEY.md Appendix A lists."""
    g10 = fixtures.case_batch("g10_deep", 900)
    assert g10["depth"].max() > 255                      # ks_shuffle rotate + truncate (A.10)
    g5 = fixtures.load_case("g05_lowdepth")
    st = harness.Setup("g05_lowdepth", ["snp", "-m", "2"], "chr1")
    assert harness.snp_oob_cells(harness.oracle_run(st))  # segbase borrow (A.3)
    g6 = fixtures.load_case("g06_softmask")
    assert any(c.islower() for c in g6["refseq"].decode())  # case-sensitive compare (A.5)
    b8 = fixtures.case_batch("g08_filters")
    assert ((b8["reads"] >> 8) & 0xFF).min() < 13        # mapQ filter
    assert (fixtures.case_batch("g12_regions")["ref"] & 0x80).sum() >= 500   # coverage gap: no callback
