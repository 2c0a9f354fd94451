"""Host pileup feeder (libpopbam_feed.so) against the fixtures' pileup restatement.

For every golden fixture the C++ feeder reads in.bam (+ .bai) and ref.fa and must produce
exactly the batch tests/golden/fixtures.build_batch derives from the same file -- the batch
whose GPU results match the reference's printed outputs (test_gpu_golden.py).  Regions are
checked against slices of the whole-contig batch (a region fetch sees the same reads at each
of its positions), with and without the index."""
import os
import shutil

import numpy as np
import pytest

import fixtures
from popbam_amd import feed
from popbam_amd import options as opt

CASES = fixtures.case_dirs()


def _feed_batch(name, max_depth, beg=None, end=None, bam_path=None):
    c = fixtures.load_case(name)
    bam = feed.Bam(bam_path or os.path.join(c["dir"], "in.bam"))
    refs = bam.refs
    seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), refs[0][0])
    sm = opt.parse_header(bam.header_text, "in.bam")
    L = len(seq)
    b, e = (0, L) if beg is None else (beg, end)
    return bam.pileup(0, b, e, seq, sm.rg2sample, sm.n, max_depth, 0 if not sm.rg2sample else -1)


def _same(ours, ref_batch, lo, hi):
    assert np.array_equal(ours["ref"], ref_batch["ref"][lo:hi])
    assert np.array_equal(ours["depth"], ref_batch["depth"][lo:hi])
    cum = np.concatenate([[0], np.cumsum(ref_batch["depth"].sum(axis=1, dtype=np.int64))])
    assert np.array_equal(ours["reads"], ref_batch["reads"][cum[lo]:cum[hi]])


def test_fasta_fetch_matches_fixture_reader():
    for name in CASES:
        c = fixtures.load_case(name)
        assert feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), c["refs"][0][0]) == c["refseq"]


def test_header_and_refs():
    for name in CASES:
        c = fixtures.load_case(name)
        bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
        assert bam.header_text == c["header"]
        assert bam.refs == [(n, ln) for n, ln in c["refs"]]
        assert bam.has_index


@pytest.mark.parametrize("name", CASES)
def test_whole_contig_batch_matches_restatement(name):
    c = fixtures.load_case(name)
    for md in sorted({255} | {int(cs["args"][cs["args"].index("-x") + 1]) for cs in c["meta"]["cases"]
                              if "-x" in cs["args"]}):
        ours = _feed_batch(name, md)
        _same(ours, fixtures.case_batch(name, md), 0, len(c["refseq"]))


@pytest.mark.parametrize("name", ["g01_base", "g08_filters", "g12_regions"])
def test_region_batches_are_slices(name, tmp_path):
    c = fixtures.load_case(name)
    full = fixtures.case_batch(name, 255)
    L = len(c["refseq"])
    rng = np.random.default_rng(5)
    spans = [(0, 1), (L - 1, L), (1000, 1000), (6990, 7610), (16383, 16385)] + \
            [tuple(sorted(rng.integers(0, L, 2))) for _ in range(6)]
    # without the index: sequential scan must select the same reads
    noidx = tmp_path / "in.bam"
    shutil.copy(os.path.join(c["dir"], "in.bam"), noidx)
    for lo, hi in spans:
        lo, hi = int(lo), int(hi)
        if hi > L:
            continue
        _same(_feed_batch(name, 255, lo, hi), full, lo, hi)
        _same(_feed_batch(name, 255, lo, hi, bam_path=str(noidx)), full, lo, hi)


def test_unknown_read_group_is_an_error(tmp_path):
    c = fixtures.load_case("g01_base")
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    sm = opt.parse_header(bam.header_text, "in.bam")
    rg2s = dict(list(sm.rg2sample.items())[1:])      # drop one read group
    with pytest.raises(feed.FeedError) as e:
        bam.pileup(0, 0, 2000, c["refseq"], rg2s, sm.n, 255, -1)
    assert e.value.code == feed.PBF_E_RG and "Problem assigning read group" in str(e.value)


@pytest.mark.parametrize("name", CASES)
def test_multithreaded_pileup_equals_sequential(name):
    """pbf_pileup_mt (region pieces walked by several threads, each with its own handle) gives
    the same batch as one sequential walk, for piece sizes down to one 64-position block and
    for a region that does not start on a block border."""
    c = fixtures.load_case(name)
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), bam.refs[0][0])
    sm = opt.parse_header(bam.header_text, "in.bam")
    fb = 0 if not sm.rg2sample else -1
    x = max(cs["max_depth"] for cs in c["meta"]["cases"])
    for beg, end in [(0, len(seq)), (37, len(seq) - 5)]:
        one = bam.pileup(0, beg, end, seq, sm.rg2sample, sm.n, x, fb)
        for threads, chunk in [(4, 64), (3, 1000), (8, 1 << 20)]:
            mt = bam.pileup(0, beg, end, seq, sm.rg2sample, sm.n, x, fb, threads=threads, chunk=chunk)
            for k in ("ref", "depth", "reads", "block_off"):
                assert np.array_equal(one[k], mt[k]), (name, beg, end, threads, chunk, k)
    bam.close()
