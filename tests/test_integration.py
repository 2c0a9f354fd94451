"""INTEGRATION.md compiled and run as printed.

`make -C oracle integ` extracts the document's c++ blocks (the pileup callback pbg_collect, the
streamed run that replaces main_<cmd>'s window loop, main_nucdiv_gpu / main_sfs_gpu /
main_ld_gpu), compiles them against the reference's own headers, links the reference's own
objects (bam_pileup, bam_index, bgzf, pop_sample, popbam with its main renamed, ...) and
libpopbam_gpu.so (oracle/integration_main.cpp).  On the GPU the binary's stdout must equal the
TSVs the reference printed for nucdiv / sfs / ld on the golden BAMs: the reference's own BAM
reading, pileup (bam_plbuf_push -> pbg_collect) and sample model feed the C-ABI."""
import os
import subprocess
import sys

import pytest

import fixtures

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "oracle", "_ref", "integ", "popbam_integ")
INC = os.path.join(REPO, "oracle", "_ref", "integ", "integration_blocks.inc")
NAMES = ("g01_base", "g02_interleaved", "g08_filters", "g10_deep")
CASES = [(nm, i) for nm in NAMES for i, cs in enumerate(fixtures.load_case(nm)["meta"]["cases"])
         if cs["args"][0] in ("nucdiv", "sfs", "ld")]


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="the reference tree is only in the build container")
def test_integration_document_compiles_as_printed(tmp_path):
    r = subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "integ"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.access(BIN, os.X_OK)
    # the compiled blocks are the document's current text
    fresh = tmp_path / "blocks.inc"
    subprocess.run([sys.executable, os.path.join(REPO, "oracle", "extract_integration.py"),
                    os.path.join(REPO, "INTEGRATION.md"), str(fresh)], check=True, capture_output=True)
    assert fresh.read_text().splitlines()[1:] == open(INC).read().splitlines()[1:]
    nm = subprocess.run(["nm", "-D", "--undefined-only", BIN], capture_output=True, text=True, check=True).stdout
    for sym in ("pbg_create", "pbg_stream_open", "pbg_stream_push", "pbg_stream_finish", "pbg_stream_text"):
        assert sym in nm, sym


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", CASES, ids=[f"{n}-{i:02d}" for n, i in CASES])
def test_integration_binary_matches_reference(gpu_lib, name, idx, tmp_path):
    assert os.access(BIN, os.X_OK), f"{BIN} missing: build it with __graft_entry__.build() where /root/reference is"
    c = fixtures.load_case(name)
    cs = c["meta"]["cases"][idx]
    # the reference's fai_load writes ref.fa.fai beside the FASTA: work on a copy
    for f in ("ref.fa", "in.bam", "in.bam.bai"):
        os.symlink(os.path.join(c["dir"], f), tmp_path / f)
    a = cs["args"]
    argv = [BIN, a[0], "-f", "ref.fa"] + list(a[1:]) + ["in.bam", cs["region"]]
    r = subprocess.run(argv, cwd=tmp_path, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    gold = fixtures.golden_text(name, cs["stdout"])
    assert r.stdout.decode() == gold, f"{a}\n{r.stdout.decode()[:400]}\n---\n{gold[:400]}"
