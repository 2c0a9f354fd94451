"""GPU parity with the CPU oracle on the HBM-resident synthetic workload (beyond fixture
sizes): the generator, the call kernel for every row width (2/4/8/16-byte rows), and the
window-statistics kernel for every statistic, on LDS-resident and workspace-resident
windows, overlapping windows, and > 65535 pairwise differences (u16 wrap)."""
import ctypes as C

import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu

SEED = 0xC0FFEE02


def _ctx(n, n_pops=2, **kw):
    from popbam_amd import _lib, workload
    params = workload.default_params(n, n_pops, **kw)
    return _lib.Context(params, 0), params


# (samples, populations): every row width (2 / 4 / 8 / 16 bytes, both ends of each width)
# and the r^2 table sizes that leave the LDS copy (2 x 13^3 > 4096 doubles at 24 samples)
SHAPES = [(12, 2), (24, 2), (24, 3), (30, 3), (48, 2), (62, 2), (64, 4), (96, 3), (126, 2)]


# pos0 1000: template-page span borders inside the keys kernel's 512-position workgroups (the
# straddle launch); 3 * 2^14 - 320: ditto, a border 320 positions in; 2^33: no border inside a
# workgroup (pos0 a multiple of 512), positions past 32 bits
@pytest.mark.parametrize("n,kw,contig,pos0", [(12, {}, 0, 1000), (12, {}, 3, 1000), (24, {"flag": 0x02}, 0, 1000),
                                               (40, {"min_baseQ": 30, "min_mapQ": 61}, 1, 1000),
                                               (64, {"max_depth": 12, "min_depth": 8}, 0, 1000),
                                               (5, {"max_depth": 300}, 2, 1000), (96, {}, 1, 1000),
                                               (24, {}, 0, 3 * 16384 - 320), (24, {}, 1, 1 << 33),
                                               (126, {}, 0, 1 << 33)])
def test_synthetic_generator_matches_oracle(gpu_lib, n, kw, contig, pos0):
    """pbg_synth_pileup = the oracle's raw generator + the host packer (call_base's per-read
    loop, libpopbam_feed.so), for every filter variant, k width, contig key and kind of
    start position."""
    import torch
    from popbam_amd import workload
    ctx, params = _ctx(n, **kw)
    nsites = 64 * 2000 + 17
    syn = workload.SynthPileup(ctx, nsites, 10, SEED, contig=contig, pos0=pos0)
    kt = np.uint8 if ctx.k_bytes == 1 else np.uint16
    k = syn.k.cpu().numpy().view(kt).reshape(-1, n)
    rq = syn.rmsq.cpu().numpy().view(np.uint32).reshape(-1, n)
    boff = syn.block_off.cpu().numpy()
    keys = syn.keys.cpu().numpy().view(np.uint16)
    ref = syn.ref.cpu().numpy()
    cpu = harness.key_batch(harness.synth_batch(SEED, pos0, pos0 + nsites, n, 10, params.max_depth, contig), params)
    assert np.array_equal(ref, cpu["ref"])
    assert np.array_equal(k, cpu["k"])
    assert np.array_equal(rq, cpu["rmsq"])
    assert np.array_equal(boff, cpu["block_off"])
    assert syn.n_keys == len(cpu["keys"]) and np.array_equal(keys[:syn.n_keys], cpu["keys"])
    # pipelined form: worst-case keys_cap, no host sync
    syn2 = workload.SynthPileup(ctx, nsites, 10, SEED, contig=contig, pos0=pos0, keys_cap=syn.max_keys)
    assert np.array_equal(syn2.keys.cpu().numpy().view(np.uint16)[:syn.n_keys], cpu["keys"])
    # too small a keys[]: flagged, nothing written past it
    from popbam_amd import _lib
    spec = syn.spec
    small = torch.zeros(64, dtype=torch.int16, device="cuda")
    rc = ctx.lib.pbg_synth_pileup(ctx.h, C.byref(spec), syn.ref.data_ptr(), syn.k.data_ptr(), syn.rmsq.data_ptr(),
                                  syn.block_off.data_ptr(), small.data_ptr(), 32, None, None)
    assert rc == 0 and ctx.lib.pbg_check(ctx.h, None) == (_lib.PBG_E_BATCH if syn.n_keys > 32 else 0)
    assert int((small[32:] != 0).sum()) == 0
    assert ctx.lib.pbg_check(ctx.h, None) == 0
    ctx.close()


@pytest.mark.parametrize("n,kw", [
    (12, {}),                                   # 2-byte rows (the benchmark shape)
    (11, {"min_snpQ": 40}),                     # more low-quality reverts (segbase borrow)
    (24, {}),                                   # 4-byte rows
    (24, {"flag": 0x02}),                       # Illumina 1.3+ qualities (-i)
    (40, {"min_baseQ": 30, "min_mapQ": 61}),    # every read filtered by mapQ: k = 0 path
    (62, {}),                                   # 8-byte rows, widest single word
    (64, {"max_depth": 12, "min_depth": 8}),    # 16-byte rows, depth filters
    (12, {"flag": 0x20}),                       # BAM_HETEROZYGOTE: heterozygotes kept
    (96, {}),                                   # two-word masks (beyond the reference's 64)
    (126, {"min_snpQ": 40}),                    # the widest 16-byte row
])
def test_call_kernel_matches_oracle(gpu_lib, n, kw):
    import torch
    from popbam_amd import workload
    ctx, params = _ctx(n, **kw)
    n_sites = 64 * max(60, 24000 // n)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + n)
    hp = workload.HotPath(ctx, syn, [(0, n_sites)], 0)
    cb = torch.zeros(n_sites * n, dtype=torch.int64, device="cuda")
    hp.call(cb=cb)
    ctx.sync_check()
    rows = hp.rows.cpu().numpy()
    cbh = cb.cpu().numpy().view(np.uint64).reshape(n_sites, n)
    batch = harness.synth_batch(SEED + n, 0, n_sites, n, 10, params.max_depth)
    ocb, types, fq, flags = harness.oracle_call(harness.oracle_params_from(params), batch)
    bad = np.nonzero((cbh != ocb).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} positions differ, first {bad[0]}: gpu {cbh[bad[0]]} oracle {ocb[bad[0]]}"
    assert np.array_equal(rows, harness.rows_from_oracle(types, flags, ctx.row_bytes))
    ctx.close()


@pytest.mark.parametrize("n,kw", [
    (12, {}),                                   # the benchmark shape
    (11, {"min_snpQ": 40}),
    (24, {"flag": 0x02}),                       # Illumina offsets: fewer kept reads
    (40, {"min_baseQ": 30, "min_mapQ": 61}),    # k = 0 everywhere: never reference-only
    (64, {"max_depth": 12, "min_depth": 8}),
    (12, {"flag": 0x20}),
    (96, {}),
    (126, {}),
])
def test_rows_only_call_matches_oracle(gpu_lib, n, kw):
    """Rows without consensus words (the statistics path): the kernel may then skip the
    likelihood of reference-only samples (class 0); the rows must still equal the oracle's."""
    import torch
    from popbam_amd import workload
    ctx, params = _ctx(n, **kw)
    n_sites = 64 * max(60, 24000 // n)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 7 * n)
    hp = workload.HotPath(ctx, syn, [(0, n_sites)], 0)
    hp.call()
    ctx.sync_check()
    rows = hp.rows.cpu().numpy()
    batch = harness.synth_batch(SEED + 7 * n, 0, n_sites, n, 10, params.max_depth)
    _, types, _, flags = harness.oracle_call(harness.oracle_params_from(params), batch)
    expect = harness.rows_from_oracle(types, flags, ctx.row_bytes)
    bad = np.nonzero(rows != expect)[0] if rows.ndim == 1 else np.nonzero((rows != expect).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first at {bad[0]}"
    ctx.close()


@pytest.mark.parametrize("n,kw,n_sites", [(12, {}, 64 * 60000), (24, {"flag": 0x02}, 64 * 20000),
                                           (96, {}, 64 * 6000), (12, {"min_snpQ": 40}, 64 * 20000)])
def test_rows_only_equals_consensus_word_call(gpu_lib, n, kw, n_sites):
    """Size-independent check of the rows-only pipeline's shortcuts (the reference-only test,
    uniform_ref, one_error_ref and their bound margins): over every position of a batch far
    larger than the oracle cases, its rows equal those of the consensus-word call, which runs
    errmod_cal + gl2cns on every task (bench.py's rows_crosscheck does the same at 50 Msites)."""
    import torch
    from popbam_amd import workload
    ctx, params = _ctx(n, **kw)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 11 * n)
    hp = workload.HotPath(ctx, syn, [(0, n_sites)], 0)
    hp.call()
    ctx.sync_check()
    fast = hp.rows.clone()
    cb = torch.zeros(n_sites * n, dtype=torch.int64, device="cuda")
    hp.call(cb=cb)
    ctx.sync_check()
    rb = ctx.row_bytes
    bad = torch.nonzero((fast.view(-1, rb) != hp.rows.view(-1, rb)).any(dim=1)).flatten()
    assert bad.numel() == 0, f"{bad.numel()} rows differ, first at {int(bad[0])}"
    ctx.close()


def _soft_mask(ref: np.ndarray, run: int, every: int) -> np.ndarray:
    """Lower-case the reference letters of positions [k * every, k * every + run)."""
    r = ref.copy()
    pos = np.arange(len(r))
    letter = np.isin(r & 0x7F, np.frombuffer(b"ACGT", np.uint8))
    m = ((pos % every) < run) & letter
    r[m] |= 0x20
    return r


@pytest.mark.parametrize("n,kw", [(12, {}), (24, {"flag": 0x02}), (12, {"min_snpQ": 40}), (20, {"flag": 0x20})])
def test_soft_masked_reference_runs_match_oracle(gpu_lib, n, kw):
    """Long lower-case reference runs (soft-masked repeats): POPBAM compares the reference
    case-sensitively (Appendix A.5), so no key matches it and every called task leaves the
    scan's reference-only test -- the scan's list fills and the rest go to call_overflow_kernel,
    which settles uniform / one-error tasks without the sort.  Rows equal the oracle's on both
    call paths."""
    import torch
    from popbam_amd import workload
    ctx, params = _ctx(n, **kw)
    n_sites = 64 * max(60, 24000 // n)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 13 * n)
    ref = _soft_mask(syn.ref.cpu().numpy(), 3000, 5000)
    syn.ref.copy_(torch.from_numpy(ref).cuda())
    hp = workload.HotPath(ctx, syn, [(0, n_sites)], 0)
    hp.call()
    ctx.sync_check()
    rows = hp.rows.cpu().numpy()
    batch = harness.synth_batch(SEED + 13 * n, 0, n_sites, n, 10, params.max_depth)
    batch["ref"] = _soft_mask(batch["ref"], 3000, 5000)
    _, types, _, flags = harness.oracle_call(harness.oracle_params_from(params), batch)
    expect = harness.rows_from_oracle(types, flags, ctx.row_bytes)
    bad = np.nonzero(rows != expect)[0] if rows.ndim == 1 else np.nonzero((rows != expect).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first at {bad[0]}"
    cb = torch.zeros(n_sites * n, dtype=torch.int64, device="cuda")
    hp.call(cb=cb)
    ctx.sync_check()
    assert np.array_equal(hp.rows.cpu().numpy(), expect)
    ctx.close()


@pytest.mark.parametrize("n,kw", [(12, {}), (24, {"flag": 0x02}), (12, {"min_snpQ": 40})])
def test_stream_soft_masked_matches_oracle(gpu_lib, n, kw):
    """The streamed run over a host batch with long lower-case reference runs: pbg_stream_push
    sees them in the host reference and has the scan settle its list mid-block (Batch::masked)
    instead of overflowing it; rows equal the oracle's and the resident (overflow-path) call's."""
    import torch
    from popbam_amd import _lib, workload
    import bench
    ctx, params = _ctx(n, **kw)
    n_sites = 64 * max(60, 24000 // n)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 17 * n)
    ref = _soft_mask(syn.ref.cpu().numpy(), 3000, 5000)
    syn.ref.copy_(torch.from_numpy(ref).cuda())
    wins = workload.reference_windows(0, n_sites, 10_000)
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS
    hp = workload.HotPath(ctx, syn, wins, stats)
    hp.step()
    ctx.sync_check()

    class A:
        window = 10_000
    cmds, keep = bench.stat_cmds(A, n, 2, 0, n_sites)
    cmds, keep = cmds[:2], keep   # nucdiv, sfs
    host = hp.to_host()
    kb = ctx.k_bytes
    with _lib.Stream(ctx, cmds, 0, n_sites, 64 * 1000) as st:
        pl = _lib.PbgPileup(n_sites, 0, host["ref"].data_ptr(), host["k"].data_ptr(), host["rmsq"].data_ptr(),
                            host["block_off"].data_ptr(), host["keys"].data_ptr())
        st.push(pl)
        st.finish()
        rows = torch.zeros_like(hp.rows)
        st.rows_into(rows.data_ptr(), rows.numel())
    assert torch.equal(rows, hp.rows)
    batch = harness.synth_batch(SEED + 17 * n, 0, n_sites, n, 10, params.max_depth)
    batch["ref"] = _soft_mask(batch["ref"], 3000, 5000)
    _, types, _, flags = harness.oracle_call(harness.oracle_params_from(params), batch)
    expect = harness.rows_from_oracle(types, flags, ctx.row_bytes)
    got = rows.cpu().numpy()
    assert np.array_equal(got, expect)
    ctx.close()


def _window_text(ctx, params, hp, cmd_id, output, windows, min_freq=1, jc=0, min_snps=10, flag_sub=False):
    """Format the GPU window outputs with the library's print_<stat> (pbg_format)."""
    from popbam_amd import _lib
    n, np_ = params.n_samples, params.n_pops
    host = {k: v.cpu().numpy() for k, v in hp.out.t.items()}
    o = _lib.PbgWindowOut()
    for k in [f for f, _ in _lib.PbgWindowOut._fields_]:
        setattr(o, k, host[k].ctypes.data)
    c = _lib.PbgCmd()
    c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq, c.jc = cmd_id, output, 10, min_snps, min_freq, jc
    c.chr_name = b"chr1"
    sn = (C.c_char_p * n)(*[f"s{i}".encode() for i in range(n)])
    pn = (C.c_char_p * np_)(*[f"p{i}".encode() for i in range(np_)])
    c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
    c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
    c.refid = b"ref"
    wb = np.array([a for a, _ in windows], np.int32)
    we = np.array([b for _, b in windows], np.int32)
    cap = 1 << 24
    buf = C.create_string_buffer(cap)
    need = C.c_size_t()
    r = ctx.lib.pbg_format(ctx.h, C.byref(c), C.byref(o), len(windows), wb.ctypes.data, we.ctypes.data, buf, cap,
                           C.byref(need))
    ctx.check(r, "pbg_format")
    return buf.value.decode()


def _oracle_text(params, types, flags, cmd_id, output, windows, min_freq=1, jc=0, min_snps=10):
    p = harness.oracle_params_from(params)
    c = harness.OrcCmd()
    n, np_ = params.n_samples, params.n_pops
    c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq, c.jc = cmd_id, output, 10, min_snps, min_freq, jc
    c.chr_name = b"chr1"
    sn = (C.c_char_p * n)(*[f"s{i}".encode() for i in range(n)])
    pn = (C.c_char_p * np_)(*[f"p{i}".encode() for i in range(np_)])
    c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
    c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
    c.refid = b"ref"
    wb = np.array([a for a, _ in windows], np.int32)
    we = np.array([b for _, b in windows], np.int32)
    cap = 1 << 24
    buf = C.create_string_buffer(cap)
    r = harness.oracle().orc_windows_from_sites(C.byref(p), C.byref(c), types.ctypes.data, flags.ctypes.data,
                                                len(windows), wb.ctypes.data, we.ctypes.data, buf, cap)
    assert r >= 0
    return buf.value.decode()


STATS = [  # (PBG_S_* flag, popbam_func_t, -o, min_freq, jc)
    (0x001, 4, 0, 1, 0), (0x002, 6, 0, 1, 0), (0x004, 5, 0, 1, 0), (0x004, 5, 0, 2, 0), (0x008, 5, 1, 1, 0),
    (0x010, 5, 2, 1, 0), (0x020, 2, 0, 1, 0), (0x040, 2, 1, 1, 0), (0x080, 1, 0, 1, 0), (0x100, 1, 1, 1, 0),
    (0x200, 1, 2, 1, 0), (0x400, 3, 0, 1, 0), (0x400, 3, 0, 1, 1),
]


@pytest.mark.parametrize("n,npops", SHAPES, ids=[f"n{a}p{b}" for a, b in SHAPES])
@pytest.mark.parametrize("layout", ["ref10kb", "overlap", "ragged"])
@pytest.mark.parametrize("stat,cmd_id,output,min_freq,jc", STATS)
def test_window_stats_match_oracle(gpu_lib, n, npops, layout, stat, cmd_id, output, min_freq, jc):
    import torch
    from popbam_amd import workload
    n_sites = 64 * 8000 if stat != 0x008 else 64 * 1600      # omega_max is O(S^3) on the oracle
    if n > 30:
        n_sites //= 2
    if n > 64:
        n_sites //= 2
    ctx, params = _ctx(n, npops)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + n)
    if layout == "ref10kb":
        wins = workload.reference_windows(0, n_sites, 10_000)
    elif layout == "overlap":
        wins = [(s, s + 1000) for s in range(0, n_sites - 1000, 500)]           # 1 kb / 500 bp step
    else:
        rng = np.random.default_rng(7)
        cuts = np.sort(rng.choice(n_sites, 40, replace=False))
        wins = [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])] + [(5, 5), (0, 1)]
    hp = workload.HotPath(ctx, syn, wins, stat, min_freq=min_freq)
    hp.opts.jc = jc
    hp.step()
    torch.cuda.synchronize()
    types, flags = harness.rows_to_sites(hp.rows.cpu().numpy(), ctx.row_bytes, n_sites, n)
    gpu = _window_text(ctx, params, hp, cmd_id, output, wins, min_freq, jc)
    orc = _oracle_text(params, types, flags, cmd_id, output, wins, min_freq, jc)
    assert gpu == orc
    ctx.close()


@pytest.mark.parametrize("n,npops", [(12, 1), (24, 3)])
def test_zns_chain_past_the_lds_list(gpu_lib, n, npops):
    """A ZnS chain longer than window_zns_kernel's LDS list capacity (at most 4096 sites): its
    workgroup leaves the compacted fast path (s_fits) for the raw masks in the list buffer while
    the r^2 table stays in LDS -- a combination no population-size setting reaches (populations
    of at most 26 samples are compacted; wider ones have tables too large for LDS).  One window
    over the whole batch beside a 10 kb one (its own workgroup, fast path), against the oracle."""
    import torch
    from popbam_amd import workload
    n_sites = 64 * 8000
    ctx, params = _ctx(n, npops)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 11 * n)
    wins = [(0, n_sites), (1000, 11_000)]
    hp = workload.HotPath(ctx, syn, wins, 0x004)
    hp.step()
    torch.cuda.synchronize()
    ns = hp.out.t["ld_snps"].cpu().numpy().reshape(len(wins), npops)
    assert ns[0].max() > 4096, "the long chain must exceed the LDS list capacity"
    types, flags = harness.rows_to_sites(hp.rows.cpu().numpy(), ctx.row_bytes, n_sites, n)
    gpu = _window_text(ctx, params, hp, 5, 0, wins)   # ld -o 0 (PBG_S_ZNS)
    orc = _oracle_text(params, types, flags, 5, 0, wins)
    assert gpu == orc
    ctx.close()


def _interleaved_params(n, npops):
    """Populations dealt round-robin over the samples (sample v -> population v % npops), so
    pairs v < u with pop(v) > pop(u) exist (the Dxy asymmetry, Appendix A.6)."""
    from popbam_amd import workload
    p = workload.default_params(n, npops)
    masks = [0] * npops
    for i in range(npops):
        p.pop_n[i] = 0
    for v in range(n):
        masks[v % npops] |= 1 << v
        p.pop_n[v % npops] += 1
    for i, m in enumerate(masks):
        p.set_pop_mask(i, m)
    return p


@pytest.mark.parametrize("n,npops,interleave", [(12, 2, True), (30, 3, True), (96, 3, True), (126, 2, True),
                                                (96, 1, False), (126, 1, False), (70, 2, False)])
@pytest.mark.parametrize("stat,cmd_id,output", [(0x001, 4, 0), (0x080, 1, 0), (0x100, 1, 1), (0x200, 1, 2),
                                                (0x400, 3, 0)])
def test_window_stats_population_layouts(gpu_lib, n, npops, interleave, stat, cmd_id, output):
    """Population layouts beside the contiguous default: interleaved populations (calc_nucdiv's
    sums then come from sample pairs, not per-site counts) and populations of more than 64
    samples (calc_nhaps' merge in LDS instead of registers), on 1 kb / 500 bp windows (few
    segregating sites: bitplanes gathered per sample) and 10 kb windows."""
    import torch
    from popbam_amd import _lib, workload
    params = _interleaved_params(n, npops) if interleave else workload.default_params(n, npops)
    ctx = _lib.Context(params, 0)
    n_sites = 64 * 2000
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 3 * n)
    wins = [(s, s + 1000) for s in range(0, n_sites - 1000, 500)] + workload.reference_windows(0, n_sites, 10_000)
    hp = workload.HotPath(ctx, syn, wins, stat)
    hp.step()
    torch.cuda.synchronize()
    types, flags = harness.rows_to_sites(hp.rows.cpu().numpy(), ctx.row_bytes, n_sites, n)
    assert _window_text(ctx, params, hp, cmd_id, output, wins) == _oracle_text(params, types, flags, cmd_id, output, wins)
    ctx.close()


@pytest.mark.parametrize("n,npops", [(12, 2), (24, 3), (64, 4), (96, 3)])
def test_u16_wrap_and_workspace_window(gpu_lib, n, npops):
    """One window over 1.28 M positions: ~25 k segregating sites (beyond LDS -> global
    workspace) and > 65535 differences per pair for some pairs at high theta."""
    import torch
    from popbam_amd import _lib, workload
    n_sites = 64 * 20000
    ctx, params = _ctx(n, npops)
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 99)
    wins = [(0, n_sites), (1000, n_sites - 3)]
    for stat, cmd_id, output in [(0x001, 4, 0), (0x200, 1, 2), (0x020, 2, 0), (0x002, 6, 0), (0x004, 5, 0),
                                 (0x400, 3, 0)]:
        hp = workload.HotPath(ctx, syn, wins, stat)
        hp.step()
        torch.cuda.synchronize()
        types, flags = harness.rows_to_sites(hp.rows.cpu().numpy(), ctx.row_bytes, n_sites, n)
        assert int((flags & 4 > 0).sum()) > 64 * 32
        assert _window_text(ctx, params, hp, cmd_id, output, wins) == _oracle_text(params, types, flags, cmd_id,
                                                                                  output, wins)
    ctx.close()


def _device_batch(kb):
    """A host key batch -> device tensors (ref, k, rmsq, block_off, keys)."""
    import torch
    L = len(kb["ref"])
    ref = torch.from_numpy(np.ascontiguousarray(kb["ref"])).cuda()
    k = np.ascontiguousarray(kb["k"]).reshape(-1)
    kd = torch.from_numpy(k if k.dtype == np.uint8 else k.view(np.int16)).cuda()
    rq = torch.from_numpy(np.ascontiguousarray(kb["rmsq"]).reshape(-1).view(np.int32)).cuda()
    boff = torch.from_numpy(np.ascontiguousarray(kb["block_off"]).astype(np.int64)).cuda()
    keys = kb["keys"] if len(kb["keys"]) else np.zeros(8, np.uint16)
    kk = torch.from_numpy(np.ascontiguousarray(keys).view(np.int16)).cuda()
    assert len(kb["block_off"]) == (L + 63) // 64 + 1
    return ref, kd, rq, boff, kk


@pytest.mark.parametrize("name", ["g01_base", "g05_lowdepth", "g06_softmask", "g07_multiallelic", "g08_filters",
                                  "g10_deep"])
def test_fixture_rows_only_and_cb_paths_match_oracle(gpu_lib, name):
    """Both call pipelines (rows only: scan / queues / fold; with consensus words: the block
    kernel) on the golden fixtures' pileups: every row equals the oracle's."""
    import torch
    import fixtures
    from popbam_amd import _lib, engine
    cs = fixtures.load_case(name)["meta"]["cases"][0]
    st = harness.Setup(name, cs["args"], cs["region"])
    params = engine.make_params(st.opts, st.sm)
    ctx = _lib.Context(params, 0)
    n = params.n_samples
    ref, kd, rq, boff, kk = _device_batch(st.kbatch)
    L = len(st.batch["ref"])
    pl = _lib.PbgPileup(L, 0, ref.data_ptr(), kd.data_ptr(), rq.data_ptr(), boff.data_ptr(), kk.data_ptr())
    rb = ctx.row_bytes
    _, types, _, flags = harness.oracle_call(harness.oracle_params_from(params), st.batch)
    expect = harness.rows_from_oracle(types, flags, rb)
    cbw = torch.zeros(L * n, dtype=torch.int64, device="cuda")
    rows0 = torch.zeros(L * rb, dtype=torch.uint8, device="cuda")
    ctx.check(ctx.lib.pbg_call_sites(ctx.h, C.byref(pl), rows0.data_ptr(), cbw.data_ptr(), None), "pbg_call_sites")
    torch.cuda.synchronize()
    cbh = cbw.cpu().numpy().view(np.uint64).reshape(L, n)
    cum = np.concatenate([[0], np.cumsum(st.batch["depth"].reshape(-1).astype(np.int64))])

    def detail(i):
        out = []
        for s_ in range(n):
            t = i * n + s_
            rr = st.batch["reads"][cum[t]:cum[t + 1]]
            out.append((s_, int(cbh[i, s_] & 0xFFFF), [(int(r & 255), int((r >> 8) & 255), int((r >> 16) & 15))
                                                       for r in rr]))
        return out

    for with_cb in (False, True):
        rows = torch.zeros(L * rb, dtype=torch.uint8, device="cuda")
        cb = torch.zeros(L * n, dtype=torch.int64, device="cuda") if with_cb else None
        ctx.check(ctx.lib.pbg_call_sites(ctx.h, C.byref(pl), rows.data_ptr(), cb.data_ptr() if with_cb else None,
                                         None), "pbg_call_sites")
        ctx.sync_check()
        got = rows.cpu().numpy().reshape(L, rb)
        exp = np.ascontiguousarray(expect).view(np.uint8).reshape(L, rb)
        bad = np.nonzero((got != exp).any(axis=1))[0]
        if bad.size:
            i = int(bad[0])
            msg = (f"cb={with_cb}: {bad.size} rows differ, first at {i}: gpu {got[i]} oracle {exp[i]} "
                   f"ref {st.batch['ref'][i]} depth {st.batch['depth'][i].tolist()}\nbad {bad[:40].tolist()}\n{detail(i)}")
            raise AssertionError(msg)
    ctx.close()


@pytest.mark.parametrize("n,npops,flag,outidx", [(12, 2, 0, 0), (24, 3, 0x40, 5), (64, 4, 0x40, 63), (11, 1, 0, 0),
                                                 (30, 5, 0, 0), (96, 3, 0x40, 90)])
def test_sfs_bins_and_theta_w(gpu_lib, n, npops, flag, outidx):
    """The SFS bins, S and theta_W = S / a1[n_pop] (north_star outputs the reference never prints;
    parity unpinned) equal the oracle's calc_sfs integers, bit for bit, for every window layout,
    with and without the outgroup flip."""
    import torch
    from popbam_amd import _lib, workload
    ctx, params = _ctx(n, npops, flag=flag)
    n_sites = 64 * 4000
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 3 * n)
    rng = np.random.default_rng(n)
    cuts = np.sort(rng.choice(n_sites, 30, replace=False))
    wins = workload.reference_windows(0, n_sites, 10_000) + [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
    wins += [(0, n_sites), (9, 9)]
    hp = workload.HotPath(ctx, syn, wins, _lib.PBG_S_SFS)
    hp.opts.outidx = outidx
    hp.step()
    ctx.sync_check()
    types, flags = harness.rows_to_sites(hp.rows.cpu().numpy(), ctx.row_bytes, n_sites, n)
    stride = ctx.sfs_stride
    nw = len(wins)
    bins = np.zeros(nw * npops * stride, np.int32)
    segp = np.zeros(nw * npops, np.int32)
    tw = np.zeros(nw * npops, np.float64)
    c = harness.OrcCmd()
    c.outidx = outidx
    wb = np.array([a for a, _ in wins], np.int32)
    we = np.array([b for _, b in wins], np.int32)
    assert harness.oracle().orc_sfs_windows(C.byref(harness.oracle_params_from(params)), C.byref(c),
                                            types.ctypes.data, flags.ctypes.data, nw, wb.ctypes.data, we.ctypes.data,
                                            stride, bins.ctypes.data, segp.ctypes.data, tw.ctypes.data) == 0
    assert np.array_equal(hp.out.t["sfs_bins"].cpu().numpy(), bins)
    assert np.array_equal(hp.out.t["seg_pop"].cpu().numpy(), segp)
    assert np.array_equal(hp.out.t["theta_w"].cpu().numpy().view(np.uint64), tw.view(np.uint64))
    assert segp.sum() > 0
    ctx.close()


@pytest.mark.parametrize("n", [12, 32, 96])
@pytest.mark.parametrize("max_depth", [255, 300])
def test_inconsistent_batch_is_reported(gpu_lib, n, max_depth):
    """pbg_call_sites on a batch whose block_off disagrees with k[] for two blocks (4 and 5):
    the kernels never read past a block's keys, write uncounted rows for exactly those blocks,
    every other block's rows are byte-identical to the clean batch's, and pbg_check reports
    PBG_E_BATCH (then clears).  n = 12 keeps the scan's info bytes in LDS (k sum checked after
    the rounds); 32 and 96 take the wide path (k sum checked before the rounds, mid-block list
    passes); max_depth 300 stores k as u16."""
    import torch
    from popbam_amd import _lib, workload
    ctx, params = _ctx(n, max_depth=max_depth)
    L = 64 * 100
    syn = workload.SynthPileup(ctx, L, 10, SEED + n)
    rb = ctx.row_bytes
    for cb in (None, torch.zeros(L * n, dtype=torch.int64, device="cuda")):
        hp = workload.HotPath(ctx, syn, [(0, L)], 0)
        hp.call(cb=cb)
        assert ctx.lib.pbg_check(ctx.h, None) == _lib.PBG_OK
        good = hp.rows.cpu().numpy().reshape(L, rb).copy()
        syn.block_off[5] += 3
        hp.rows.fill_(0xAB)
        hp.call(cb=cb)
        assert ctx.lib.pbg_check(ctx.h, None) == _lib.PBG_E_BATCH
        assert ctx.lib.pbg_check(ctx.h, None) == _lib.PBG_OK
        bad = hp.rows.cpu().numpy().reshape(L, rb)
        assert not bad[4 * 64:6 * 64].any(), "the corrupted blocks' rows must be uncounted (0)"
        assert np.array_equal(bad[:4 * 64], good[:4 * 64]) and np.array_equal(bad[6 * 64:], good[6 * 64:])
        assert good[4 * 64:6 * 64].any()
        syn.block_off[5] -= 3
    ctx.close()


@pytest.mark.parametrize("n,npops,pieces", [(12, 2, 4), (24, 3, 3), (96, 3, 5)])
def test_pipelined_pieces_equal_one_step(gpu_lib, n, npops, pieces):
    """bench.py's pipelined steps (the contig's call in pieces at window borders, each piece's
    statistics on a second stream beside the next piece's call, across steps too) write the
    same rows and the same window outputs, byte for byte, as one call + one statistics launch."""
    import torch
    from popbam_amd import _lib, workload
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS
    ctx, params = _ctx(n, npops)
    n_sites = 2_000_000 + 37
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + n)
    wins = workload.reference_windows(0, n_sites, 10_000)
    one = workload.HotPath(ctx, syn, wins, stats)
    one.step()
    ctx.sync_check()
    two = workload.HotPath(ctx, syn, wins, stats)
    pts = two.pipeline(pieces)
    assert len(pts) == pieces + 1 and all(p % 64 == 0 for p in pts[:-1])
    s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream()
    for _ in range(3):   # back-to-back steps: the last piece's statistics overlap the next first call
        two.step_pipelined(s1, s2)
    torch.cuda.synchronize()
    ctx.sync_check()
    assert torch.equal(one.rows, two.rows)
    for k in workload.HotPath.fields_for(stats):
        assert torch.equal(one.out.t[k].view(torch.uint8), two.out.t[k].view(torch.uint8)), k
    assert int(one.out.t["segsites"].sum()) > 0
    ctx.close()


@pytest.mark.parametrize("n,npops,pinned,chunk", [(12, 2, True, 64 * 2000), (12, 2, False, 64 * 3000),
                                                  (32, 2, True, 0), (96, 3, False, 64 * 700)])
def test_stream_equals_resident(gpu_lib, n, npops, pinned, chunk):
    """The C-ABI streamed run (pbg_stream_open / _push / _finish): the batch handed over in HOST
    memory -- pinned (DMA straight from the caller's buffers) or pageable (threaded copy into the
    context's pinned staging) -- in several pieces, each split into device chunks that alternate
    between two slots, gives the resident step's rows bit for bit and its nucdiv / sfs / ld text
    byte for byte, twice in a row on the same context (slots, window lists and plans reused).
    The keys pointer of each chunk is shifted back to the chunk's first key, so the kernels must
    read only keys [block_off[0], block_off[last]) (include/popbam_gpu.h)."""
    import torch
    from popbam_amd import _lib, workload
    import bench
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS
    ctx, params = _ctx(n, npops)
    n_sites = 1_000_000 + 37
    syn = workload.SynthPileup(ctx, n_sites, 10, SEED + 7 * n)
    wins = workload.reference_windows(0, n_sites, 10_000)
    hp = workload.HotPath(ctx, syn, wins, stats)
    hp.step()
    ctx.sync_check()

    class A:
        window = 10_000
    cmds, keep = bench.stat_cmds(A, n, npops, 0, n_sites)
    want = bench.resident_texts(ctx, hp, cmds, wins)
    host = hp.to_host()
    if not pinned:
        host = {k: v.clone() for k, v in host.items()}   # pageable copies
        assert not host["keys"].is_pinned()
    kb = ctx.k_bytes
    cuts = [0, 64 * 3001, 64 * 9000, n_sites]   # three pieces: multiples of 64 but the last
    for _ in range(2):
        with _lib.Stream(ctx, cmds, 0, n_sites, chunk) as st:
            for a, b in zip(cuts[:-1], cuts[1:]):
                pl = _lib.PbgPileup(b - a, a, host["ref"].data_ptr() + a, host["k"].data_ptr() + a * n * kb,
                                    host["rmsq"].data_ptr() + a * n * 4, host["block_off"].data_ptr() + (a // 64) * 8,
                                    host["keys"].data_ptr())
                st.push(pl)
            st.finish()
            rows = torch.zeros_like(hp.rows)
            st.rows_into(rows.data_ptr(), rows.numel())
            assert torch.equal(rows, hp.rows)
            assert [st.text(i) for i in range(3)] == want
            prof = st.profile()
            assert prof["pieces"] == 3 and prof["chunks"] >= 3
            assert (prof["pinned_chunks"] == prof["chunks"]) == pinned
    ctx.close()
