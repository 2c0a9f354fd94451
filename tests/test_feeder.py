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


def _py_pack(batch, n, min_baseQ, min_mapQ, illumina):
    """numpy restatement of call_base's per-read loop (popbam.cpp:252-287) for the check."""
    r = batch["reads"].astype(np.int64)
    raw = r & 0xFF
    bq = np.where(raw > 31, raw - 31, 0) if illumina else raw
    mq = (r >> 8) & 0xFF
    nt = (r >> 16) & 0xF
    ok = (bq >= (min_baseQ & 0xFF)) & (mq >= (min_mapQ & 0xFF)) & np.isin(nt, [1, 2, 4, 8])
    base = np.select([nt == 1, nt == 2, nt == 4], [0, 1, 2], 3)
    qq = np.clip(np.minimum(bq, mq), 4, 63)
    key = (qq << 5) | (((r >> 20) & 1) << 4) | base
    task = np.repeat(np.arange(batch["depth"].size), batch["depth"].reshape(-1).astype(np.int64))
    k = np.bincount(task[ok], minlength=batch["depth"].size)
    rmsq = np.bincount(task[ok], weights=(mq * mq)[ok], minlength=batch["depth"].size).astype(np.int64)
    return k.reshape(-1, n), rmsq.reshape(-1, n), key[ok].astype(np.uint16)


@pytest.mark.parametrize("name", CASES)
def test_key_batches(name):
    """pbf_pileup_keys_mt (pileup + partition + call_base's per-read loop, threaded) equals
    pbf_pack of the restated raw batch, and pbf_pack equals a numpy restatement of the loop,
    for the filter settings the case's commands use."""
    c = fixtures.load_case(name)
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), bam.refs[0][0])
    sm = opt.parse_header(bam.header_text, "in.bam")
    fb = 0 if not sm.rg2sample else -1
    seen = set()
    for cs in c["meta"]["cases"]:
        o = opt.parse_args(cs["args"][0], list(cs["args"][1:]) + ["in.bam", "chr1"])
        key = (o.min_baseQ & 0xFF, o.min_mapQ & 0xFF, o.flag & 0x02, o.max_depth)
        if key in seen:
            continue
        seen.add(key)
        flt = feed.make_filter(o.min_baseQ, o.min_mapQ, o.flag, o.max_depth)
        raw = fixtures.case_batch(name, o.max_depth)
        packed = feed.pack(raw, sm.n, flt)
        k, rmsq, keys = _py_pack(raw, sm.n, o.min_baseQ, o.min_mapQ, o.flag & 0x02)
        assert np.array_equal(packed["k"], k) and np.array_equal(packed["rmsq"], rmsq)
        assert np.array_equal(packed["keys"], keys) and np.array_equal(packed["ref"], raw["ref"])
        cum = np.concatenate([[0], np.cumsum(k.sum(axis=1))])
        assert np.array_equal(packed["block_off"], cum[::64] if len(k) % 64 == 0 else
                              np.concatenate([cum[::64], cum[-1:]]))
        for threads, chunk in [(1, 1 << 20), (4, 64), (3, 1000)]:
            mt = bam.pileup_keys(0, 0, len(seq), seq, sm.rg2sample, sm.n, o.max_depth, flt, fb, threads=threads,
                                 chunk=chunk)
            for f in ("ref", "k", "rmsq", "keys", "block_off"):
                assert np.array_equal(mt[f], packed[f]), (name, key, threads, f)
    bam.close()


def test_pack_rejects_wide_k_in_u8():
    raw = fixtures.case_batch("g10_deep", 900)
    with pytest.raises(feed.FeedError):
        feed.pack(raw, raw["depth"].shape[1], feed.make_filter(13, 13, 0, 255))
    wide = feed.pack(raw, raw["depth"].shape[1], feed.make_filter(13, 13, 0, 900))
    assert wide["k"].dtype == np.uint16 and wide["k"].max() > 255


def _crowded_bam(tmp_path):
    """A pile deep enough for the pileup buffer's maxcnt (8000 reads, bam_pileup.c:375): 4000
    reads on [60, 110) then 4100 on [100, 160), two samples, so which reads at 100 are kept
    depends on whether the walk started before 110 (it then still holds the first pile)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from bamwriter import Read, write_bam
    L = 400
    reads = []
    for i in range(8100):
        pos, ln = (60, 50) if i < 4000 else (100, 60)
        reads.append(Read(f"r{i}", 0, pos, 40, 16 * (i & 1), [("M", ln)], "ACGT" * (ln // 4) + "A" * (ln % 4),
                          [30 + i % 7] * ln, {"RG": f"rg{i & 1}"}))
    hdr = "@HD\tVN:1.0\tSO:coordinate\n@SQ\tSN:chr1\tLN:%d\n" % L
    hdr += "".join(f"@RG\tID:rg{s}\tSM:s{s}\tPO:p{s}\n" for s in range(2))
    path = str(tmp_path / "crowd.bam")
    write_bam(path, hdr, [("chr1", L)], reads)
    return path, ("ACGT" * (L // 4)).encode(), {"rg0": 0, "rg1": 1}


def test_crowded_pileup_follows_the_reference_walks(tmp_path):
    """Where the maxcnt drop depends on where a walk starts, pbf_pileup_mt gives what the
    reference's own walks give: one fresh fetch + walk per window (pop_nucdiv.cpp:57-125), or
    one walk of the region without windows -- for every piece size."""
    path, seq, rg2s = _crowded_bam(tmp_path)
    bam = feed.Bam(path)
    beg, end, X = 0, 320, 20000

    def reference_walks(win):
        if win == 0:
            return bam.pileup(0, beg, end, seq, rg2s, 2, X, -1)
        depth, reads = [], []
        a = beg
        while a < end:
            k = (a - beg) // win
            wb, we = beg + k * win, beg + k * win + win - 1
            sa, sb = (wb, min(we, end)) if a < we else (a, a + 1)
            part = bam.pileup(0, sa, sb, seq, rg2s, 2, X, -1)
            depth.append(part["depth"][a - sa:])
            skip = int(part["depth"][:a - sa].sum())
            reads.append(part["reads"][skip:])
            a = sb
        return {"depth": np.concatenate(depth), "reads": np.concatenate(reads)}

    seen = set()
    for win in (0, 64, 100, 37):
        want = reference_walks(win)
        seen.add(int(want["depth"][130].sum()))
        for threads, chunk in [(1, 64), (3, 64), (2, 128), (4, 1 << 20)]:
            got = bam.pileup(0, beg, end, seq, rg2s, 2, X, -1, threads=max(2, threads), chunk=chunk, win=win)
            assert np.array_equal(got["depth"], want["depth"]), (win, threads, chunk)
            assert np.array_equal(got["reads"], want["reads"]), (win, threads, chunk)
    assert len(seen) > 1   # the fixture does reach maxcnt differently per walk start
    bam.close()


def test_crowded_key_batches_follow_the_reference_walks(tmp_path):
    """The key path (pbf_pileup_keys_mt / pbf_kstream_*: records parsed into an arena, one walk
    per piece) falls back to the reference's window-by-window walks where a read can meet a full
    buffer (maxcnt): its keys equal pbf_pack of the raw reference walks for every window size."""
    path, seq, rg2s = _crowded_bam(tmp_path)
    bam = feed.Bam(path)
    beg, end, X = 0, 320, 20000
    flt = feed.make_filter(13, 13, 0, X)
    for win in (0, 64, 37):
        raw = bam.pileup(0, beg, end, seq, rg2s, 2, X, -1, threads=2, chunk=64, win=win)
        want = feed.pack(raw, 2, flt)
        for threads, chunk in [(1, 64), (3, 128), (2, 1 << 20)]:
            got = bam.pileup_keys(0, beg, end, seq, rg2s, 2, X, flt, -1, threads=threads, chunk=chunk, win=win)
            for f in ("ref", "k", "rmsq", "keys", "block_off"):
                assert np.array_equal(got[f], want[f]), (win, threads, chunk, f)
    bam.close()


def test_key_stream_pieces_concatenate_to_the_batch():
    """pbf_kstream_next hands out the pieces in position order; concatenated they are the
    merged batch (pbf_pileup_keys_mt), and the profile counts the inflated bytes and records."""
    c = fixtures.load_case("g16_24s2p")
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), bam.refs[0][0])
    sm = opt.parse_header(bam.header_text, "in.bam")
    flt = feed.make_filter(13, 13, 0, 255)
    beg, end = 100, len(seq) - 3
    whole = bam.pileup_keys(0, beg, end, seq, sm.rg2sample, sm.n, 255, flt, -1, threads=3, chunk=1000)
    parts = []
    with bam.key_stream(0, beg, end, seq, sm.rg2sample, sm.n, 255, flt, -1, threads=4, chunk=640) as ks:
        while True:
            p = ks.next()
            if p is None:
                break
            parts.append(feed._take_keys(bam.lib, p, sm.n, 1))
        prof = ks.profile()
    assert [p["pos0"] for p in parts] == list(range(beg, end, 640))
    assert np.array_equal(np.concatenate([p["keys"] for p in parts]), whole["keys"])
    assert np.array_equal(np.concatenate([p["k"] for p in parts]), whole["k"])
    assert np.array_equal(np.concatenate([p["ref"] for p in parts]), whole["ref"])
    assert prof["pieces"] == len(parts) and prof["bytes_inflated"] > prof["bytes_compressed"] > 0
    assert prof["records"] > 0 and prof["t_inflate"] <= prof["t_fetch"]
    bam.close()


def test_key_path_unknown_read_group_is_an_error():
    c = fixtures.load_case("g01_base")
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    sm = opt.parse_header(bam.header_text, "in.bam")
    rg2s = dict(list(sm.rg2sample.items())[1:])      # drop one read group
    with pytest.raises(feed.FeedError) as e:
        bam.pileup_keys(0, 0, 2000, c["refseq"], rg2s, sm.n, 255, feed.make_filter(13, 13, 0, 255), -1, threads=2,
                        chunk=640)
    assert e.value.code == feed.PBF_E_RG and "Problem assigning read group" in str(e.value)
    bam.close()


def test_zlib_and_libdeflate_inflate_alike(tmp_path):
    """BGZF blocks inflate to the same records with libdeflate and with zlib's inflate (the
    fallback, POPBAM_NO_LIBDEFLATE=1): the key batch is identical."""
    import subprocess
    import sys
    code = ("import sys, numpy as np; sys.path[:0] = [%r, %r]; import fixtures, os\n"
            "from popbam_amd import feed, options as opt\n"
            "c = fixtures.load_case('g11_eleven'); bam = feed.Bam(os.path.join(c['dir'], 'in.bam'))\n"
            "seq = feed.fasta_fetch(os.path.join(c['dir'], 'ref.fa'), bam.refs[0][0]); sm = opt.parse_header(bam.header_text, 'in.bam')\n"
            "b = bam.pileup_keys(0, 0, len(seq), seq, sm.rg2sample, sm.n, 255, feed.make_filter(13, 13, 0, 255), -1, threads=2, chunk=4096)\n"
            "np.save(sys.argv[1], b['keys'])\n") % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    outs = []
    for env in ({}, {"POPBAM_NO_LIBDEFLATE": "1"}):
        p = str(tmp_path / f"k{len(outs)}.npy")
        subprocess.run([sys.executable, "-c", code, p], check=True, env=dict(os.environ, **env))
        outs.append(np.load(p))
    assert len(outs[0]) > 0 and np.array_equal(outs[0], outs[1])


def _python_synth_bam(d, seed, L, n, npops=2, read_len=100, step=10):
    """The record-by-record writer the native one (oracle/synth_bam.cpp) replaced: the same reads
    through tests/golden/bamwriter.py."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import harness
    from bamwriter import Read, write_bam, write_fasta
    os.makedirs(d, exist_ok=True)
    lib = harness.oracle()
    lib.orc_synth_genotypes.restype = None
    lib.orc_synth_genotypes.argtypes = [C.c_uint64, C.c_int32, C.c_uint64, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p]
    ref = np.zeros(L, np.uint8)
    al = np.zeros((L, n), np.uint8)
    lib.orc_synth_genotypes(seed, 0, 0, L, n, ref.ctypes.data, al.ctypes.data)
    bases = np.frombuffer(b"ACGT", np.uint8)
    per = n // npops
    header = ["@HD\tVN:1.0\tSO:coordinate", f"@SQ\tSN:chr1\tLN:{L}"]
    header += [f"@RG\tID:rg{s}\tSM:s{s}\tPO:pop{min(s // per, npops - 1)}" for s in range(n)]
    reads = []
    for s in range(n):
        for i, p in enumerate(range(s % step, L - read_len + 1, step)):
            h = (i + s) & 1
            seq = bases[(al[p:p + read_len, s] >> (2 * h)) & 3].tobytes().decode()
            reads.append(Read(name=f"r{s}_{i}", tid=0, pos=p, mapq=60, flag=16 if (i >> 1) & 1 else 0,
                              cigar=[("M", read_len)], seq=seq, qual=[40] * read_len, tags={"RG": f"rg{s}"}))
    reads.sort(key=lambda r: r.pos)
    write_fasta(os.path.join(d, "ref.fa"), [("chr1", ref.tobytes().decode())])
    write_bam(os.path.join(d, "in.bam"), "\n".join(header) + "\n", [("chr1", L)], reads)


def test_native_synthetic_bam_equals_python_writer(tmp_path):
    """oracle/synth_bam.cpp (the CPU baseline's and the command-line benchmark's BAM) holds the
    same header, reference and reads as the Python writer's file, and POPBAM itself prints the
    same text on both."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import ref_baseline
    L, n = 30_000, 12
    a, b = str(tmp_path / "native"), str(tmp_path / "python")
    ref_baseline.make_inputs(a, 0xC0FFEE02, L, n)
    _python_synth_bam(b, 0xC0FFEE02, L, n)
    assert open(os.path.join(a, "ref.fa")).read() == open(os.path.join(b, "ref.fa")).read()
    batches = []
    for d in (a, b):
        bam = feed.Bam(os.path.join(d, "in.bam"))
        assert bam.has_index and bam.refs == [("chr1", L)]
        sm = opt.parse_header(bam.header_text, "in.bam")
        seq = feed.fasta_fetch(os.path.join(d, "ref.fa"), "chr1")
        batches.append((bam.header_text, bam.pileup_keys(0, 0, L, seq, sm.rg2sample, sm.n, 255,
                                                         feed.make_filter(13, 13, 0, 255), -1, threads=2, chunk=5000)))
        # a region fetch through the index (linear index + bins)
        part = bam.pileup_keys(0, 17_000, 23_000, seq, sm.rg2sample, sm.n, 255, feed.make_filter(13, 13, 0, 255), -1)
        full = batches[-1][1]
        lo, hi = int(full["k"][:17_000].sum()), int(full["k"][:23_000].sum())
        assert np.array_equal(part["k"], full["k"][17_000:23_000]) and np.array_equal(part["keys"], full["keys"][lo:hi])
        bam.close()
    assert batches[0][0] == batches[1][0]
    for f in ("ref", "k", "rmsq", "keys", "block_off"):
        assert np.array_equal(batches[0][1][f], batches[1][1][f]), f
    if ref_baseline.available():
        outs = [subprocess.run([ref_baseline.REF_BIN, "nucdiv", "-f", "ref.fa", "-w", "5", "in.bam", "chr1:2001-27000"],
                               cwd=d, capture_output=True, check=True).stdout for d in (a, b)]
        assert outs[0] == outs[1] and outs[0].count(b"\n") >= 4


def test_kstream_error_is_sticky():
    """A failing piece (a read group no sample owns: the reference's fatal 'Problem assigning read
    group', popbam.cpp:234-240) is reported by pbf_kstream_next, and again by every later call
    instead of a wait for a piece that never comes."""
    import concurrent.futures as cf
    c = fixtures.load_case("g01_base")
    bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
    seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), bam.refs[0][0])
    flt = feed.make_filter(13, 13, 0, 255)
    ks = bam.key_stream(0, 0, len(seq), seq, {}, 12, 255, flt, -1, threads=2, chunk=4096)
    with ks:
        codes = []
        for _ in range(3):
            with cf.ThreadPoolExecutor(1) as ex:
                fut = ex.submit(ks.next)
                try:
                    fut.result(timeout=20)
                    codes.append(0)
                except feed.FeedError as e:
                    codes.append(e.code)
        assert codes == [feed.PBF_E_RG] * 3
