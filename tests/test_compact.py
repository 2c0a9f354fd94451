"""Compact pieces (pbg_stream_push_compact, pbf_filter.compact, pbf_compact): a reference-only task
-- 1..32 keys, every key on the upper-case A/C/G/T reference base of a called position, the
scan's own reference-only test (call_kernel.hip call_scan_kernel) -- crosses the boundary with
rmsq bit 31 set and without its keys (the streamed C-ABI was PCIe-bound on
keys of tasks the scan settles from k and sum mapQ^2 alone).

CPU: the compact form follows that definition task by task; the feeder's compact pieces (the
walk flags while it packs) equal the full pieces compacted afterwards.  GPU: a streamed run of
compact pieces gives the rows and the TSV text of the full pieces (and of the resident step) at
12 / 24 / 96 samples, soft-masked references included; a flag on a task that cannot be
reference-only is an error, not a silent wrong row."""
import os

import numpy as np
import pytest

import fixtures
import harness
from popbam_amd import feed
from popbam_amd import options as opt

SEED = 0xC0FFEE21


def _reference_only(keys, n):
    """The definition, task by task, on a full key batch (numpy, no library)."""
    ref = keys["ref"]
    k = keys["k"].reshape(-1).astype(np.int64)
    base_of = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}
    off = np.concatenate([[0], np.cumsum(k)]) + int(keys["block_off"][0])
    out = np.zeros(k.size, bool)
    for t in range(k.size):
        c = int(ref[t // n])
        if c & 0x80 or c not in base_of or not 1 <= k[t] <= 32:
            continue
        out[t] = bool(np.all((keys["keys"][off[t]:off[t + 1]] & 3) == base_of[c]))
    return out


def _soft(ref, lo, hi):
    r = ref.copy()
    m = (r >= ord("A")) & (r <= ord("Z"))
    r[lo:hi][m[lo:hi]] |= 0x20
    return r


@pytest.mark.parametrize("n", [12, 24])
def test_compact_form_follows_the_definition(n):
    from popbam_amd import workload
    params = workload.default_params(n)
    L = 64 * 150 + 17
    batch = harness.synth_batch(SEED + n, 0, L, n, 10, params.max_depth)
    batch["ref"] = _soft(batch["ref"], 2000, 2600)      # lower-case run: nothing flagged there
    batch["ref"][3000:3100] |= 0x80                     # positions without a callback
    full = harness.key_batch(batch, params)
    kb = 1 if params.max_depth <= 255 else 2
    cmp = feed.compact(full, n, kb)
    want = _reference_only(full, n)
    flag = (cmp["rmsq"].reshape(-1) >> 31).astype(bool)
    assert np.array_equal(flag, want)
    assert 0.85 < want.mean() < 0.97                    # most tasks: depth 10, 1/128 errors
    assert np.array_equal(cmp["rmsq"].reshape(-1) & 0x7FFFFFFF, full["rmsq"].reshape(-1))
    assert np.array_equal(cmp["k"], full["k"]) and np.array_equal(cmp["ref"], full["ref"])
    # the unflagged tasks' keys, in order; block_off counts them
    k = full["k"].reshape(-1).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(k)])
    kept = np.concatenate([full["keys"][off[t]:off[t + 1]] for t in np.nonzero(~want)[0]] or [np.zeros(0, np.uint16)])
    assert np.array_equal(cmp["keys"], kept)
    pres = np.where(want, 0, k)
    nb = (L + 63) // 64
    blk = np.concatenate([[0], np.cumsum([pres[b * 64 * n:(b + 1) * 64 * n].sum() for b in range(nb)])])
    assert np.array_equal(cmp["block_off"][:nb + 1], blk)
    assert cmp["keys"].size < 0.2 * full["keys"].size


def test_feeder_compact_pieces_equal_compacted_full_pieces():
    """The walk's own flagging (fast walk and, for crowded pieces, pbf_pack) = pbf_compact of the
    full pieces, piece for piece, on golden BAMs."""
    for name in ("g01_base", "g16_24s2p", "g06_softmask"):
        c = fixtures.load_case(name)
        bam = feed.Bam(os.path.join(c["dir"], "in.bam"))
        seq = feed.fasta_fetch(os.path.join(c["dir"], "ref.fa"), bam.refs[0][0])
        sm = opt.parse_header(bam.header_text, "in.bam")
        full = bam.pileup_keys(0, 0, len(seq), seq, sm.rg2sample, sm.n, 255, feed.make_filter(13, 13, 0, 255), -1,
                               threads=2, chunk=1280)
        cmp = bam.pileup_keys(0, 0, len(seq), seq, sm.rg2sample, sm.n, 255, feed.make_filter(13, 13, 0, 255, True), -1,
                              threads=2, chunk=1280)
        want = feed.compact(full, sm.n, 1)
        for f in ("ref", "k", "rmsq", "keys", "block_off"):
            assert np.array_equal(cmp[f], want[f]), (name, f)
        assert (cmp["rmsq"] >> 31).any()
        bam.close()


def _stream(ctx, cmds, n_sites, host, compact, chunk):
    import torch
    from popbam_amd import _lib
    n, kb = ctx.params.n_samples, ctx.k_bytes
    cuts = [0] + [c for c in (64 * 1001, 64 * 4000) if c < n_sites] + [n_sites]
    with _lib.Stream(ctx, cmds, 0, n_sites, chunk) as st:
        for a, b in zip(cuts[:-1], cuts[1:]):
            pl = _lib.PbgPileup(b - a, a, host["ref"][a:].ctypes.data, host["k"].reshape(-1)[a * n:].ctypes.data,
                                host["rmsq"].reshape(-1)[a * n:].ctypes.data,
                                host["block_off"][a // 64:].ctypes.data, host["keys"].ctypes.data)
            st.push(pl, compact=compact)
        st.finish()
        rows = torch.zeros(n_sites * ctx.row_bytes, dtype=torch.uint8, device="cuda")
        st.rows_into(rows.data_ptr(), rows.numel())
        texts = [st.text(i) for i in range(len(cmds))]
        prof = st.profile()
    return rows, texts, prof


@pytest.mark.gpu
@pytest.mark.parametrize("n,npops,soft", [(12, 2, False), (12, 2, True), (24, 3, False), (96, 3, True)])
def test_compact_stream_equals_full_stream(gpu_lib, n, npops, soft):
    import torch
    from popbam_amd import _lib, workload
    import bench
    params = workload.default_params(n, npops)
    ctx = _lib.Context(params, 0)
    n_sites = 64 * 6000 + 29
    batch = harness.synth_batch(SEED + 3 * n, 0, n_sites, n, 10, params.max_depth)
    if soft:
        batch["ref"] = _soft(batch["ref"], 50_000, 58_000)
    full = harness.key_batch(batch, params)
    kb = ctx.k_bytes
    cmp = feed.compact(full, n, kb)

    class A:
        window = 10_000
    cmds, keep = bench.stat_cmds(A, n, npops, 0, n_sites)
    rows_f, texts_f, prof_f = _stream(ctx, cmds, n_sites, full, False, 64 * 1500)
    rows_c, texts_c, prof_c = _stream(ctx, cmds, n_sites, cmp, True, 64 * 1500)
    ctx.sync_check()
    assert torch.equal(rows_f, rows_c)
    assert texts_f == texts_c
    assert prof_c["h2d_bytes"] < 0.5 * prof_f["h2d_bytes"]
    _, types, _, flags = harness.oracle_call(harness.oracle_params_from(params), batch)
    expect = harness.rows_from_oracle(types, flags, ctx.row_bytes)
    got = rows_c.cpu().numpy().view(expect.dtype).reshape(expect.shape)
    assert np.array_equal(got, expect)
    ctx.close()


@pytest.mark.gpu
def test_compact_flag_on_a_variant_task_is_an_error(gpu_lib):
    """A producer that flags a task which is not reference-only (here: one at a lower-case
    reference position, its keys taken out as a flagged task's are) gets PBG_E_BATCH from
    pbg_stream_finish with the compact message, not rows that silently differ."""
    from popbam_amd import _lib, workload
    import bench
    n = 12
    params = workload.default_params(n)
    ctx = _lib.Context(params, 0)
    n_sites = 64 * 200
    batch = harness.synth_batch(SEED + 99, 0, n_sites, n, 10, params.max_depth)
    batch["ref"] = _soft(batch["ref"], 1000, 1200)
    full = harness.key_batch(batch, params)
    cmp = feed.compact(full, n, 1)
    # a task at position 1100 (lower-case: never flagged) with 1..32 keys: drop its keys, flag it
    k = cmp["k"].reshape(-1).astype(np.int64)
    rq = cmp["rmsq"].reshape(-1)
    pres = np.where(rq >> 31, 0, k)
    t = next(t for t in range(1100 * n, 1101 * n) if 1 <= k[t] <= 32)
    off = np.concatenate([[0], np.cumsum(pres)])
    keys = np.delete(cmp["keys"], np.arange(off[t], off[t + 1]))
    rq = rq.copy()
    rq[t] |= np.uint32(0x80000000)
    pres[t] = 0
    nb = (n_sites + 63) // 64
    boff = np.concatenate([[0], np.cumsum([pres[b * 64 * n:(b + 1) * 64 * n].sum() for b in range(nb)])]).astype(np.uint64)
    bad = dict(cmp, keys=keys, rmsq=rq.reshape(cmp["rmsq"].shape), block_off=np.concatenate([boff, boff[-1:]]))

    class A:
        window = 10_000
    cmds, keep = bench.stat_cmds(A, n, 2, 0, n_sites)
    with pytest.raises(RuntimeError) as e:
        _stream(ctx, cmds[:1], n_sites, bad, True, 0)
    assert "compact piece flagged" in str(e.value)
    ctx.close()
