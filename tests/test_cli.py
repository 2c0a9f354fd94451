"""The drop-in command line (popbam_amd/cli.py): `popbam <cmd> -f ref.fa [opts] in.bam region`
read with the native feeder and computed on the GPU must print exactly what the compiled
reference printed for every golden case (tests/golden/*/meta.json records the reference's
argv: make_golden.py ran `popbam <cmd> -f ref.fa <args...> in.bam <region>`).  The error
paths (fatal_error, pop_utils.cpp:510-519) need no GPU."""
import os
import shutil

import pytest

import fixtures
import harness
from popbam_amd import cli

CASES = harness.all_cases()


def _argv(name, cs):
    d = fixtures.load_case(name)["dir"]
    a = cs["args"]
    return [a[0], "-f", os.path.join(d, "ref.fa")] + list(a[1:]) + [os.path.join(d, "in.bam"), cs["region"]]


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", CASES, ids=[f"{n}-{i:02d}" for n, i in CASES])
def test_cli_matches_reference(gpu_lib, name, idx):
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    argv = _argv(name, cs)
    ours = cli.run(argv[0], argv[1:])
    gold = fixtures.golden_text(name, cs["stdout"])
    oob = None
    if cs["args"][0] == "snp":
        st = harness.Setup(name, cs["args"], cs["region"])
        oob = harness.snp_oob_cells(harness.oracle_run(st))
    ok, diff = harness.same_output(cs["args"], gold, ours, oob)
    assert ok, f"{argv}\n gold: {diff[0]}\n ours: {diff[1]}"


SHARD_CASES = [("g13_snpformats", 3), ("g13_snpformats", 5), ("g01_base", 0), ("g15_24s3p", 2), ("g12_regions", 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_cli_rank_blocks_concatenate_to_reference(gpu_lib, world):
    """cli.run(rank=r, world=W) for every r, concatenated in rank order, is the reference's
    output (window blocks, snp -o 2 header printed once with the run's total)."""
    for name, idx in SHARD_CASES:
        cases = fixtures.load_case(name)["meta"]["cases"]
        cs = cases[min(idx, len(cases) - 1)]
        argv = _argv(name, cs)
        ours = "".join(cli.run(argv[0], argv[1:], rank=r, world=world) for r in range(world))
        gold = fixtures.golden_text(name, cs["stdout"])
        oob = None
        if cs["args"][0] == "snp":
            oob = harness.snp_oob_cells(harness.oracle_run(harness.Setup(name, cs["args"], cs["region"])))
        ok, diff = harness.same_output(cs["args"], gold, ours, oob)
        assert ok, f"{argv} world={world}\n gold: {diff[0]}\n ours: {diff[1]}"


@pytest.mark.gpu
def test_cli_popbam_world_two_processes(gpu_lib):
    """POPBAM_WORLD=2: two rank processes (both on GPU 0 here), text gathered to rank 0 over gloo."""
    import subprocess
    import sys
    name = "g13_snpformats"
    cs = [c for c in fixtures.load_case(name)["meta"]["cases"] if c["args"] == ["snp", "-o", "2", "-w", "2"]][0]
    argv = _argv(name, cs)
    env = dict(os.environ, POPBAM_WORLD="2")
    r = subprocess.run([sys.executable, "-m", "popbam_amd.cli", *argv], env=env, capture_output=True, timeout=100,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr.decode()
    gold = fixtures.golden_text(name, cs["stdout"])
    oob = harness.snp_oob_cells(harness.oracle_run(harness.Setup(name, cs["args"], cs["region"])))
    ok, diff = harness.same_output(cs["args"], gold, r.stdout.decode(), oob)
    assert ok, diff


def test_cli_popbam_world_reports_rank_errors(tmp_path):
    """A sharded run whose ranks fail before the GPU: rank 0 reports the error, status 1, no hang."""
    import subprocess
    import sys
    d = fixtures.load_case("g01_base")["dir"]
    env = dict(os.environ, POPBAM_WORLD="2")
    r = subprocess.run([sys.executable, "-m", "popbam_amd.cli", "nucdiv", "-f", os.path.join(d, "ref.fa"),
                        os.path.join(d, "in.bam"), "chrX:1-100"], env=env, capture_output=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 1 and r.stdout == b""
    assert r.stderr.decode().count("Bad genome coordinates: chrX:1-100") == 1


def test_cli_popbam_world_reports_gpu_side_errors():
    """A rank failing after the options are parsed, on the library side (pbg_create refuses
    device 99: PbgError, not a PopbamError) still reaches the gather: status 1, one message,
    no hang (only PopbamError used to be caught)."""
    import subprocess
    import sys
    d = fixtures.load_case("g01_base")["dir"]
    env = dict(os.environ, POPBAM_WORLD="2", POPBAM_DEVICE="99")
    r = subprocess.run([sys.executable, "-m", "popbam_amd.cli", "nucdiv", "-f", os.path.join(d, "ref.fa"), "-w", "1",
                        os.path.join(d, "in.bam"), "chr1"], env=env, capture_output=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 1 and r.stdout == b"", r.stderr.decode()
    err = r.stderr.decode()
    assert err.count("popbam runtime error:") == 1 and "PbgError" in err


def test_negative_max_depth_is_refused(capsys):
    d = fixtures.load_case("g01_base")["dir"]
    rc, out, err = _main(["nucdiv", "-f", os.path.join(d, "ref.fa"), "-x", "-5", os.path.join(d, "in.bam"), "chr1"],
                         capsys)
    assert rc == 1 and out == "" and "-x -5 must not be negative" in err


BLOCK_CASES = [c for c in CASES if "-w" in fixtures.load_case(c[0])["meta"]["cases"][c[1]]["args"]
               and c[0] in ("g01_base", "g12_regions", "g13_snpformats", "g11_eleven")]


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", BLOCK_CASES, ids=[f"{n}-{i:02d}" for n, i in BLOCK_CASES])
def test_cli_block_streaming_matches_reference(gpu_lib, name, idx, monkeypatch):
    """POPBAM_BLOCK_SITES of two windows: the region runs as many blocks (the next block's
    pileup read while the GPU runs this one, snp -o 2's header only in the first block) and
    the concatenated text is still the reference's."""
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    a = cs["args"]
    w = int(a[a.index("-w") + 1]) * 1000
    monkeypatch.setenv("POPBAM_BLOCK_SITES", str(2 * w))
    argv = _argv(name, cs)
    ours = cli.run(argv[0], argv[1:])
    gold = fixtures.golden_text(name, cs["stdout"])
    oob = None
    if a[0] == "snp":
        oob = harness.snp_oob_cells(harness.oracle_run(harness.Setup(name, a, cs["region"])))
    ok, diff = harness.same_output(a, gold, ours, oob)
    assert ok, f"{argv}\n gold: {diff[0]}\n ours: {diff[1]}"


def _main(argv, capsys):
    rc = cli.main(argv)
    out = capsys.readouterr()
    return rc, out.out, out.err


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", [c for c in CASES if c[0] in ("g01_base", "g08_filters", "g10_deep", "g13_snpformats",
                                                                  "g16_24s2p") and c[1] < 3])
def test_cli_small_feeder_pieces_match_reference(gpu_lib, name, idx, monkeypatch):
    """64-position feeder pieces on 3 worker threads: every piece is its own pbg_stream_push (two
    device slots alternating, keys pointers shifted per chunk), and stdout is still the
    reference's byte for byte."""
    monkeypatch.setenv("POPBAM_FEED_CHUNK", "64")
    monkeypatch.setenv("POPBAM_FEED_THREADS", "3")
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    argv = _argv(name, cs)
    ours = cli.run(argv[0], argv[1:])
    oob = None
    if cs["args"][0] == "snp":
        st = harness.Setup(name, cs["args"], cs["region"])
        oob = harness.snp_oob_cells(harness.oracle_run(st))
    ok, diff = harness.same_output(cs["args"], fixtures.golden_text(name, cs["stdout"]), ours, oob)
    assert ok, f"{argv}\n gold: {diff[0]}\n ours: {diff[1]}"
    assert cli.last_profile["gpu"]["pieces"] >= 1


def test_usage_and_unknown_commands(capsys):
    rc, out, err = _main([], capsys)
    assert rc == 1 and "Usage:" in err and out == ""
    rc, out, err = _main(["frobnicate"], capsys)
    assert rc == 1 and err == "Error: unrecognized command: frobnicate\n"
    rc, out, err = _main(["tree", "x.bam", "chr1"], capsys)
    assert rc == 1 and "Cannot read BAM file x.bam" in err


def test_fatal_errors_before_the_gpu(capsys, tmp_path):
    d = fixtures.load_case("g01_base")["dir"]
    ref, bam = os.path.join(d, "ref.fa"), os.path.join(d, "in.bam")
    rc, out, err = _main(["nucdiv", "-f", ref, str(tmp_path / "missing.bam"), "chr1"], capsys)
    assert rc == 1 and out == "" and err.startswith("popbam runtime error:\nCannot read BAM file")
    assert err.endswith("Exiting program\n")
    rc, out, err = _main(["nucdiv", "-f", ref, bam, "chrX:1-100"], capsys)
    assert rc == 1 and "Bad genome coordinates: chrX:1-100" in err
    rc, out, err = _main(["nucdiv", "-f", ref, bam], capsys)
    assert rc == 1 and "Need to specify BAM file name" in err
    rc, out, err = _main(["diverge", "-f", ref, "-d", "kimura", bam, "chr1"], capsys)
    assert rc == 1 and "kimura is not a valid distance option" in err
    rc, out, err = _main(["tree", "-f", ref, "-d", "kimura", bam, "chr1"], capsys)
    assert rc == 1 and "kimura is not a valid distance option" in err
    noidx = tmp_path / "in.bam"
    shutil.copy(bam, noidx)
    rc, out, err = _main(["nucdiv", "-f", ref, str(noidx), "chr1"], capsys)
    assert rc == 1 and f"Index file not available for BAM file {noidx}" in err
    rc, out, err = _main(["nucdiv", "-f", str(tmp_path / "none.fa"), bam, "chr1"], capsys)
    assert rc == 1 and "Failed to load index for fastA reference file" in err


THETA_CASES = [("g01_base", 1), ("g03_threepops", 1), ("g04_outgroup", 0), ("g12_regions", 2), ("g15_24s3p", 22),
               ("g18_64s4p", 15), ("g01_base", 18)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", THETA_CASES, ids=[f"{n}-{i:02d}" for n, i in THETA_CASES])
def test_cli_sfs_theta_extension(gpu_lib, name, idx):
    """`popbam sfs --theta` (an extension: calc_sfs, pop_sfs.cpp:246-263, computes S and the
    spectrum but print_sfs never prints them): the reference's columns stay byte-identical and
    the appended S[p] / thetaW[p] / sfs[p] columns are consistent: S = sum of bins 1..n-1 and
    theta_W = S / a1[n] (calc_a1, pop_sfs.cpp:511-525).  The bins themselves are pinned against
    the oracle's calc_sfs integers by test_gpu_scale.py::test_sfs_bins_and_theta_w."""
    import re
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    argv = _argv(name, cs)
    ours = cli.run(argv[0], argv[1:] + ["--theta"])
    gold = fixtures.golden_text(name, cs["stdout"])
    lines, glines = ours.splitlines(), gold.splitlines()
    assert len(lines) == len(glines) and lines
    seen = 0
    for ln, gl in zip(lines, glines):
        assert ln.startswith(gl + "\tS["), (gl, ln)
        ext = ln[len(gl):].split("\t")[1:]
        assert len(ext) % 6 == 0
        for j in range(0, len(ext), 6):
            pop = re.fullmatch(r"S\[(.+)\]:", ext[j]).group(1)
            assert ext[j + 2] == f"thetaW[{pop}]:" and ext[j + 4] == f"sfs[{pop}]:"
            s = int(ext[j + 1])
            bins = [int(b) for b in ext[j + 5].split(",")]
            n = len(bins) - 1
            assert s == sum(bins[1:n]) and min(bins) >= 0
            a1 = sum(1.0 / i for i in range(1, n))
            if ext[j + 3].strip() == "NA":
                assert n < 2
            else:
                assert abs(float(ext[j + 3]) - s / a1) <= 5e-6, (ext[j + 3], s, a1)
            seen += s
    assert seen > 0
