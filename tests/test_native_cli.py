"""The native host binary `bin/popbam` (popbam_amd/csrc/popbam_main.cpp): the drop-in command as
users run it -- one fresh process per command, as the reference (popbam.cpp:53-77 dispatch ->
main_<cmd>).  Every golden case must print exactly what the compiled reference printed
(tests/golden/*/meta.json holds the reference's argv); the error paths (fatal_error,
pop_utils.cpp:510-519) must match the Python command line's messages and need no GPU."""
import os
import subprocess

import pytest

import fixtures
import harness
from popbam_amd import cli

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "bin", "popbam")
NATIVE = os.path.join(REPO, "popbam_amd", "popbam")
CASES = harness.all_cases()


def _argv(name, cs):
    d = fixtures.load_case(name)["dir"]
    a = cs["args"]
    return [a[0], "-f", os.path.join(d, "ref.fa")] + list(a[1:]) + [os.path.join(d, "in.bam"), cs["region"]]


def _run(argv, env=None, timeout=120):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    r = subprocess.run([BIN, *argv], capture_output=True, timeout=timeout, env=e)
    return r.returncode, r.stdout.decode(), r.stderr.decode()


def _oob(name, cs):
    if cs["args"][0] != "snp":
        return None
    return harness.snp_oob_cells(harness.oracle_run(harness.Setup(name, cs["args"], cs["region"])))


def test_native_binary_is_built_and_links_only_the_c_abis():
    """The binary exists, uses libpopbam_gpu.so + libpopbam_feed.so through their C-ABIs and
    nothing of Python or torch."""
    assert os.access(NATIVE, os.X_OK), "build it with __graft_entry__.build()"
    r = subprocess.run(["readelf", "-d", NATIVE], capture_output=True, text=True, check=True)
    needed = [ln.split("[")[1].rstrip("]") for ln in r.stdout.splitlines() if "(NEEDED)" in ln]
    assert "libpopbam_gpu.so" in needed and "libpopbam_feed.so" in needed
    assert not any("python" in x or "torch" in x for x in needed), needed


def test_native_usage_and_unknown_command():
    rc, out, err = _run([])
    assert rc == 1 and "Usage:" in err and out == ""
    rc, out, err = _run(["frobnicate"])
    assert rc == 1 and err == "Error: unrecognized command: frobnicate\n"


def test_native_fatal_errors_match_the_python_cli(tmp_path, capsys):
    d = fixtures.load_case("g01_base")["dir"]
    ref, bam = os.path.join(d, "ref.fa"), os.path.join(d, "in.bam")
    noidx = tmp_path / "in.bam"
    noidx.write_bytes(open(bam, "rb").read())
    cases = [["nucdiv", "-f", ref, str(tmp_path / "missing.bam"), "chr1"],
             ["nucdiv", "-f", ref, bam, "chrX:1-100"],
             ["nucdiv", "-f", ref, bam],
             ["diverge", "-f", ref, "-d", "kimura", bam, "chr1"],
             ["tree", "-f", ref, "-d", "kimura", bam, "chr1"],
             ["ld", "-f", ref, "-o", "7", bam, "chr1"],
             ["nucdiv", "-f", ref, str(noidx), "chr1"],
             ["nucdiv", "-f", str(tmp_path / "none.fa"), bam, "chr1"],
             ["nucdiv", "-f", ref, "-x", "-5", bam, "chr1"],
             ["sfs", "-f", ref, "-p", "nobody", bam, "chr1"]]
    for argv in cases:
        rc, out, err = _run(argv)
        prc = cli.main(argv)
        pe = capsys.readouterr()
        assert rc == prc == 1 and out == "" == pe.out, argv
        assert err == pe.err, (argv, err, pe.err)


def test_native_world_reports_rank_errors_once():
    """POPBAM_WORLD=2 forks two ranks; both fail before the GPU: one message, status 1."""
    d = fixtures.load_case("g01_base")["dir"]
    rc, out, err = _run(["nucdiv", "-f", os.path.join(d, "ref.fa"), os.path.join(d, "in.bam"), "chrX:1-100"],
                        env={"POPBAM_WORLD": "2"})
    assert rc == 1 and out == ""
    assert err.count("Bad genome coordinates: chrX:1-100") == 1 and err.count("popbam runtime error:") == 1


def test_native_option_conversions_follow_getopt_pp():
    """GetOpt_pp converts through std::stringstream (getopt_pp.h:133-144): the native parser uses the
    same conversions, so a bad value leaves what the extraction wrote (A.12).  Checked through the
    parse error paths only (no GPU): '-o 3' is out of range for ld, '-o 2x' converts to 2 (valid:
    the run proceeds to the region check), '-o x' converts to 0, '-o 1.5' to 1."""
    d = fixtures.load_case("g01_base")["dir"]
    ref, bam = os.path.join(d, "ref.fa"), os.path.join(d, "in.bam")
    rc, _, err = _run(["ld", "-f", ref, "-o", "3", bam, "chrX"])
    assert rc == 1 and "Not a valid output option" in err
    for v in ("2x", "x", "1.5"):
        rc, _, err = _run(["ld", "-f", ref, "-o", v, bam, "chrX"])
        assert rc == 1 and "Bad genome coordinates: chrX" in err, (v, err)


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", CASES, ids=[f"{n}-{i:02d}" for n, i in CASES])
def test_native_binary_matches_reference(gpu_lib, name, idx):
    """A fresh `bin/popbam` process per golden case: stdout byte-identical to the reference's."""
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    rc, out, err = _run(_argv(name, cs))
    assert rc == 0, err
    ok, diff = harness.same_output(cs["args"], fixtures.golden_text(name, cs["stdout"]), out, _oob(name, cs))
    assert ok, f"{cs['args']}\n gold: {diff[0]}\n ours: {diff[1]}"


NATIVE_SHARD = [("g13_snpformats", 3), ("g13_snpformats", 5), ("g01_base", 0), ("g15_24s3p", 2), ("g12_regions", 1),
                ("g01_base", 21)]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_native_world_ranks_concatenate_to_reference(gpu_lib, world):
    """POPBAM_WORLD=N: N forked rank processes (all on GPU 0 here), blocks printed in rank order."""
    for name, idx in NATIVE_SHARD:
        cases = fixtures.load_case(name)["meta"]["cases"]
        cs = cases[min(idx, len(cases) - 1)]
        rc, out, err = _run(_argv(name, cs), env={"POPBAM_WORLD": str(world)})
        assert rc == 0, err
        ok, diff = harness.same_output(cs["args"], fixtures.golden_text(name, cs["stdout"]), out, _oob(name, cs))
        assert ok, f"{cs['args']} world={world}\n gold: {diff[0]}\n ours: {diff[1]}"


SMALL = [c for c in CASES if c[0] in ("g01_base", "g08_filters", "g10_deep", "g13_snpformats") and c[1] < 4]


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx", SMALL, ids=[f"{n}-{i:02d}" for n, i in SMALL])
def test_native_small_pieces_and_blocks_match_reference(gpu_lib, name, idx):
    """64-position feeder pieces on 3 threads and blocks of two windows: many pushes, many
    streams per process, and still the reference's stdout."""
    cs = fixtures.load_case(name)["meta"]["cases"][idx]
    env = {"POPBAM_FEED_CHUNK": "64", "POPBAM_FEED_THREADS": "3"}
    a = cs["args"]
    if "-w" in a:
        env["POPBAM_BLOCK_SITES"] = str(2 * int(a[a.index("-w") + 1]) * 1000)
    rc, out, err = _run(_argv(name, cs), env=env)
    assert rc == 0, err
    ok, diff = harness.same_output(a, fixtures.golden_text(name, cs["stdout"]), out, _oob(name, cs))
    assert ok, f"{a}\n gold: {diff[0]}\n ours: {diff[1]}"


@pytest.mark.gpu
def test_native_profile_phases(gpu_lib, tmp_path):
    """POPBAM_PROFILE=<file>: one JSON line of the process's phases (bench.py's `cli` breakdown)."""
    import json
    name = "g01_base"
    cs = fixtures.load_case(name)["meta"]["cases"][0]
    prof = tmp_path / "prof.jsonl"
    rc, out, err = _run(_argv(name, cs), env={"POPBAM_PROFILE": str(prof)})
    assert rc == 0, err
    p = json.loads(prof.read_text().splitlines()[-1])["popbam_profile"]
    for k in ("parse_s", "fasta_s", "hip_init_s", "pbg_create_s", "walk_push_s", "finish_s", "run_s"):
        assert k in p and p[k] >= 0, k
    assert p["blocks"] == 1 and p["gpu"]["chunks"] >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("fault_at", [1, 2, 5, 40])
def test_native_push_failure_exits_cleanly(gpu_lib, fault_at):
    """A failing pbg_stream_push (POPBAM_FAULT_PUSH=k: the k-th push of the run reports an error)
    ends the process like fatal_error -- the message, "Exiting program", status 1 -- whether the
    failing piece was one taken while the GPU context was built (the others then still owned by
    the run) or one of the walk's later pieces: no double free, no abort."""
    name = "g01_base"
    cs = fixtures.load_case(name)["meta"]["cases"][0]
    rc, out, err = _run(_argv(name, cs), env={"POPBAM_FAULT_PUSH": str(fault_at), "POPBAM_FEED_CHUNK": "64",
                                              "POPBAM_FEED_THREADS": "3"})
    if rc == 0:   # fewer pushes than fault_at: the run is the reference's
        assert fault_at > 2, err
        return
    assert rc == 1, (rc, err)
    assert "popbam runtime error:" in err and "pbg_stream_push failed" in err and "Exiting program" in err
    assert out == ""
