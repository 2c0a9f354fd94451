"""More than 64 samples (BASELINE configs[4]: 96 samples; SURVEY 8(f) 3: multi-word rows).

The reference stops at 64 samples (u64 masks, popbam.cpp:168), so no reference output exists
beyond.  The oracle runs the same algorithm on 128-bit masks; it is pinned here by embedding
the 64-sample golden case g18_64s4p into 96 samples: the four original populations keep their
order and their samples' order, a fifth population of copies of samples 0..31 is inserted
after the second, so populations 2 and 3 move into the masks' second word.  Copies call
exactly as their originals, so the counted and segregating positions do not change, and every
statistic below that depends on a population's own samples (and, for dxy, on the order of two
populations' samples) equals the reference's golden value for that population.

Not invariant under the embedding, so compared only GPU-vs-oracle (test_gpu_* below):
Wall's B/Q (last_type is shared across populations, Appendix A.9, and the copies are
variable wherever populations 0/1 are) and snp (one column per sample).
"""
import numpy as np
import pytest

import fixtures
import harness

CASE = "g18_64s4p"
INVARIANT = [a for a in (c["args"] for c in fixtures.load_case(CASE)["meta"]["cases"])
             if not (a[0] == "snp" or (a[0] == "ld" and "-o" in a and a[a.index("-o") + 1] == "2"))]


def _golden(args):
    for c in fixtures.load_case(CASE)["meta"]["cases"]:
        if c["args"] == args:
            return fixtures.golden_text(CASE, c["stdout"]), c["region"]
    raise KeyError(args)


@pytest.mark.parametrize("args", INVARIANT, ids=[" ".join(a) for a in INVARIANT])
def test_wide_oracle_reproduces_the_reference_on_embedded_populations(args):
    gold, region = _golden(args)
    st = harness.WideSetup(CASE, args, region)
    assert st.sm.n == 96 and max(i for i, p in enumerate(st.sm.sample_pop) if p == 4) == 95
    ours = harness.oracle_run(st)
    g, o = harness.labelled_values(gold), harness.labelled_values(ours)
    assert len(gold.splitlines()) == len(ours.splitlines())
    missing = [k for k in g if k not in o]
    assert not missing, missing[:5]
    bad = [(k, g[k], o[k]) for k in g if g[k] != o[k]]
    assert not bad, bad[:5]
    # the inserted population is reported too (its own columns exist)
    assert any("[copies]" in k[1] for k in o) or args[0] == "diverge" and "-o" not in args


def test_select_samples_regroups_reads():
    b = harness.synth_batch(5, 0, 640, 6, 10)
    sel = harness.select_samples(b, [3, 0, 3])
    assert sel["depth"].shape == (640, 3)
    assert np.array_equal(sel["depth"][:, 0], b["depth"][:, 3]) and np.array_equal(sel["depth"][:, 2], b["depth"][:, 3])
    cum = np.concatenate([[0], np.cumsum(b["depth"].reshape(-1).astype(np.int64))])
    cs = np.concatenate([[0], np.cumsum(sel["depth"].reshape(-1).astype(np.int64))])
    for i in (0, 17, 639):
        for j, s in enumerate([3, 0, 3]):
            a = b["reads"][cum[i * 6 + s]:cum[i * 6 + s + 1]]
            assert np.array_equal(sel["reads"][cs[i * 3 + j]:cs[i * 3 + j + 1]], a)


def test_wide_calls_split_into_independent_samples():
    """96-sample calls = the calls of each half on its own (a sample's consensus word reads
    only its reads); the 96-bit type mask is the halves' masks side by side, a position is
    counted iff both halves are, and segregating iff counted with exactly one derived allele
    across all 96 samples (segbase, pop_utils.cpp:122-168)."""
    from popbam_amd import workload
    n, L = 96, 64 * 300
    b = harness.synth_batch(0xABCD, 0, L, n, 10)
    p96 = harness.oracle_params_from(workload.default_params(n, 3))
    cb, types, fq, flags = harness.oracle_call(p96, b)
    assert types.shape == (L, 2)
    halves = []
    for lo in (0, 48):
        part = harness.select_samples(b, list(range(lo, lo + 48)))
        halves.append(harness.oracle_call(harness.oracle_params_from(workload.default_params(48, 1)), part))
    assert np.array_equal(cb, np.concatenate([halves[0][0], halves[1][0]], axis=1))
    t0, t1 = halves[0][1].astype(object), halves[1][1].astype(object)
    both = ((flags & 2) > 0)
    assert np.array_equal(both, ((halves[0][3] & 2) > 0) & ((halves[1][3] & 2) > 0))
    wide = types[:, 0].astype(object) | (types[:, 1].astype(object) << 64)
    assert all(wide[i] == (t0[i] | (t1[i] << 48)) for i in np.nonzero(both)[0])
    # segregating: counted, and the derived samples carry one allele (genotype byte of cb)
    g = (cb >> np.uint64(8)) & np.uint64(0xFF)
    der = (cb & np.uint64(3)) == np.uint64(3)
    allele = (g >> np.uint64(2)) & np.uint64(3)
    for i in np.nonzero(both)[0][:2000]:
        al = set(allele[i][der[i]].tolist())
        assert bool(flags[i] & 4) == (len(al) == 1), i
    assert int((flags & 4 > 0).sum()) > 50


GPU_ARGS = [c["args"] for c in fixtures.load_case(CASE)["meta"]["cases"]] + [
    ["snp", "-o", "1"], ["snp", "-o", "2", "-w", "1"], ["tree", "-w", "1"], ["tree", "-w", "1", "-d", "jc"]]


@pytest.mark.gpu
@pytest.mark.parametrize("copies", [32, 62])
@pytest.mark.parametrize("args", GPU_ARGS, ids=[" ".join(a) for a in GPU_ARGS])
def test_gpu_wide_run_matches_wide_oracle(gpu_lib, args, copies):
    """pbg_run (key batch -> call kernels -> statistics -> TSV) with 96 and 126 samples: the
    whole text equals the 128-bit oracle's (pinned above), Wall and snp included."""
    from popbam_amd import engine
    st = harness.WideSetup(CASE, args, "chr1", n_copies=copies)
    assert st.sm.n == 64 + copies
    ours = engine.run_command(st.opts, st.sm, st.chr, st.beg, st.end, st.kbatch, refid=st.refid)
    orc = harness.oracle_run(st)
    oob = harness.snp_oob_cells(orc) if args[0] == "snp" else None
    ok, diff = harness.same_output(args, orc, ours, oob)
    assert ok, f"{args}: {diff}"
