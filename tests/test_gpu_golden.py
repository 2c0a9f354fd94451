"""GPU parity against the reference's own outputs: every golden case run through the C-ABI
(pbg_run -> call kernel -> window-statistics kernel -> TSV writer) must print exactly what
the compiled reference printed on the same BAM.  snp base cells where the reference reads
out of bounds (UB, Appendix A.3) are masked using the oracle's marks."""
import pytest

import fixtures
import harness
from popbam_amd import engine

CASES = harness.all_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", CASES, ids=[f"{n}-{i:02d}" for n, i in CASES])
def test_gpu_matches_reference(gpu_lib, name, idx):
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    st = harness.Setup(name, cs["args"], cs["region"])
    ours = engine.run_command(st.opts, st.sm, st.chr, st.beg, st.end, st.kbatch, refid=st.refid)
    gold = fixtures.golden_text(name, cs["stdout"])
    oob = harness.snp_oob_cells(harness.oracle_run(st)) if cs["args"][0] == "snp" else None
    ok, diff = harness.same_output(cs["args"], gold, ours, oob)
    assert ok, f"{cs['args']} {cs['region']}\n gold: {diff[0]}\n ours: {diff[1]}"


@pytest.mark.gpu
def test_ms_header_needs_a_window(gpu_lib):
    """snp -o 2 prints its header inside the window loop at cw == 0 (pop_snp.cpp:114-115): a
    region shorter than one window prints nothing at all (oracle and GPU agree; no golden case
    can hold an empty output, parity pinned by the reference's loop structure)."""
    st = harness.Setup("g13_snpformats", ["snp", "-o", "2", "-w", "2"], "chr1:1-1500")
    assert harness.oracle_run(st) == ""
    assert engine.run_command(st.opts, st.sm, st.chr, st.beg, st.end, st.kbatch, refid=st.refid) == ""
    st = harness.Setup("g13_snpformats", ["snp", "-o", "2", "-w", "2"], "chr1:1-2001")   # one window: header
    ours = engine.run_command(st.opts, st.sm, st.chr, st.beg, st.end, st.kbatch, refid=st.refid)
    assert ours.startswith("ms ") and ours == harness.oracle_run(st)
