"""Whole-genome pass (popbam_amd.genome, configs[3]): the contig-first shard plan covers every
window exactly once, and the chunked, double-buffered pass -- pileup generated chunk by chunk
on one stream, called on another, rows kept genome-resident -- gives the same rows and the same
window statistics, byte for byte, as one batch per contig."""
import numpy as np
import pytest

from popbam_amd import genome, workload

SEED = 0xC0FFEE04


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8, 16, 30])
@pytest.mark.parametrize("lengths,win", [([125_000_000] * 24, 10_000), ([30_017, 1_000_000, 64, 250_001], 1_000),
                                         ([5_000_000], 10_000), ([999, 10_001, 20_000], 1_000)])
def test_plan_covers_every_window_once(world, lengths, win):
    plan = genome.plan_genome(lengths, world, win)
    assert len(plan) == world
    got = {}
    for segs in plan:
        for s in segs:
            for a, b in genome.contig_windows(s.end, win, s.beg, s.end):
                key = (s.contig, a, b)
                assert key not in got
                got[key] = True
            assert 0 <= s.beg < s.end <= lengths[s.contig]
    want = {(ci, a, b) for ci, L in enumerate(lengths) for a, b in genome.contig_windows(L, win)}
    assert set(got) == want
    loads = [sum(s.end - s.beg for s in segs) for segs in plan]
    if world <= len(lengths):
        assert max(loads) <= 2 * (sum(lengths) / world) + max(win, max(lengths) // world + win)


@pytest.mark.gpu
@pytest.mark.parametrize("n,npops", [(12, 2), (24, 2)])
def test_chunked_pass_equals_one_batch(gpu_lib, n, npops):
    import torch
    from popbam_amd import _lib
    ctx = _lib.Context(workload.default_params(n, npops), 0)
    lengths = [640_017, 1_000_000, 300_000]
    segs = [genome.Segment(i, 0, L) for i, L in enumerate(lengths)] + [genome.Segment(1, 250_000, 700_001)]
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS | _lib.PBG_S_DIV_IND
    small = genome.GenomePass(ctx, segs, SEED, 10, 10_000, stats, chunk=64 * 2000)
    small.run()
    small.run()   # a second pass over the same buffers gives the same result
    small.synchronize()
    big = genome.GenomePass(ctx, segs, SEED, 10, 10_000, stats, chunk=64 * 20000)
    big.run()
    big.synchronize()
    assert len(small.chunks) > len(big.chunks)
    for si, s in enumerate(segs):
        a = small.segment_rows(si).cpu().numpy()
        b = big.segment_rows(si).cpu().numpy()
        assert np.array_equal(a, b), si
        # one batch of the segment through the plain hot path
        syn = workload.SynthPileup(ctx, s.end - s.beg, 10, SEED, contig=s.contig, pos0=s.beg)
        wins = [(x - s.beg, y - s.beg) for x, y in genome.contig_windows(s.end, 10_000, s.beg, s.end)]
        hp = workload.HotPath(ctx, syn, wins or [(0, 0)], stats)
        hp.step()
        ctx.sync_check()
        assert np.array_equal(hp.rows.cpu().numpy(), a), si
    for f in workload.HotPath.fields_for(stats):
        x, y = small.window_results(f), big.window_results(f)
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), f
    # the window outputs of the last segment against its one-batch hot path
    nw = len(wins)
    for f in ("pi", "td", "ld_val", "div_ind", "theta_w", "sfs_bins"):
        per = hp.out.t[f].numel() // max(1, len(wins))
        tail = small.window_results(f)[-nw * per:]
        assert np.array_equal(tail.view(np.uint8), hp.out.t[f][:nw * per].cpu().numpy().view(np.uint8)), f
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,config", [(24, 3), (96, 4)])
def test_serial_pass_equals_double_buffered(gpu_lib, n, config):
    """GenomePass(serial=True) -- each chunk generated on the call stream right before its call,
    one buffer: the mode bench.py times by default -- writes the same rows, window outputs and
    key_total as the double-buffered pass, over two passes."""
    from popbam_amd import _lib
    ctx = _lib.Context(workload.default_params(n, 2), 0)
    if config == 3:
        segs = [genome.Segment(0, 0, 700_001), genome.Segment(2, 100_000, 400_017)]
        stats, win = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS | _lib.PBG_S_DIV_IND, 10_000
    else:
        segs = genome.plan_overlapping(300_000, 1, 1000, 500)[0]
        stats, win = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_HAP_EHHS, 1000
    got = []
    for serial in (True, False):
        gp = genome.GenomePass(ctx, segs, SEED + n, 10, win, stats, chunk=64 * 1500, serial=serial)
        for _ in range(2):
            gp.run()
        gp.synchronize()
        got.append((gp.rows.cpu().numpy(), {f: gp.window_results(f) for f in workload.HotPath.fields_for(stats)},
                    int(gp.key_total.item())))
    assert np.array_equal(got[0][0], got[1][0])
    for f in got[0][1]:
        assert np.array_equal(got[0][1][f].view(np.uint8), got[1][1][f].view(np.uint8)), f
    assert got[0][2] == got[1][2] > 0
    ctx.close()


@pytest.mark.parametrize("world", [1, 2, 3, 8, 13])
@pytest.mark.parametrize("length,win,step", [(200_000_000, 1000, 500), (10_007, 1000, 500), (5_000, 700, 300),
                                             (999, 1000, 500)])
def test_overlapping_plan_covers_every_window_once(world, length, win, step):
    """configs[4]'s overlapping windows: contiguous window blocks per rank, each segment holds
    its windows entirely (the halo of win - step positions included), and every window
    [k*step, k*step + win) of the contig lands on exactly one rank."""
    plan = genome.plan_overlapping(length, world, win, step)
    assert len(plan) == world
    got = []
    for segs in plan:
        for s in segs:
            ws = list(range(s.win_lo, s.win_hi, s.step))
            assert ws and s.beg == ws[0] and s.end == ws[-1] + win <= length
            got += ws
    want = list(range(0, length - win + 1, step)) if length >= win else []
    assert got == want


@pytest.mark.gpu
def test_overlapping_pass_matches_one_batch(gpu_lib):
    """96 samples, overlapping 1 kb windows every 500 bp, nucdiv + sfs + haplo EHHS: the chunked
    pass over a two-rank plan equals one batch of the whole contig through the hot path."""
    from popbam_amd import _lib
    n, L, win, step = 96, 400_000, 1000, 500
    ctx = _lib.Context(workload.default_params(n, 2), 0)
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_HAP_EHHS
    parts = []
    for segs in genome.plan_overlapping(L, 2, win, step):
        gp = genome.GenomePass(ctx, segs, SEED, 10, win, stats, chunk=64 * 1000)
        gp.run()
        gp.synchronize()
        parts.append(gp)
    syn = workload.SynthPileup(ctx, L, 10, SEED, contig=0, pos0=0)
    wins = [(a, a + win) for a in range(0, L - win + 1, step)]
    hp = workload.HotPath(ctx, syn, wins, stats)
    hp.step()
    ctx.sync_check()
    for f in workload.HotPath.fields_for(stats):
        x = np.concatenate([p.window_results(f) for p in parts])
        assert np.array_equal(x.view(np.uint8), hp.out.t[f].cpu().numpy().view(np.uint8)), f
    assert (hp.out.t["segsites"].cpu().numpy() > 0).mean() > 0.5
    ctx.close()


def _rank_plan_worker(rank, world, port, results):
    """One gloo rank: its bench_genome split (genome.rank_plan) for configs[3] and configs[4],
    gathered on rank 0 over gloo (the only collective the bench uses, on the host)."""
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = {}
        for config, lengths, win, step in ((3, [125_000_000] * 24, 10_000, 0), (4, [200_000_000], 1000, 500)):
            segs, stats = genome.rank_plan(config, lengths, world, rank, win, step)
            mine[config] = ([(s.contig, s.beg, s.end, s.step, s.win_lo, s.win_hi) for s in segs], stats)
        got = [None] * world
        dist.all_gather_object(got, mine)
        if rank == 0:
            results.update({r: got[r] for r in range(world)})
    finally:
        dist.destroy_process_group()


def test_gloo_world8_rank_split_covers_genome():
    """bench.py's N = 8 split, run as 8 gloo processes: configs[3] windows land on exactly one
    rank each with per-rank loads within one window of the mean (24 equal contigs over 8 ranks:
    3 whole contigs each); configs[4]'s overlapping-window blocks tile the window list in rank
    order, each with its win - step halo."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 8
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_rank_plan_worker, args=(world, port, results), nprocs=world, join=True)
    res = [results[r] for r in range(world)]
    lengths, win = [125_000_000] * 24, 10_000
    seen = set()
    loads = []
    for r in range(world):
        segs, stats = res[r][3]
        assert stats == res[0][3][1]
        loads.append(sum(e - b for _, b, e, *_ in segs))
        for ci, b, e, *_ in segs:
            for w in genome.contig_windows(e, win, b, e):
                assert (ci, w) not in seen
                seen.add((ci, w))
    assert seen == {(ci, w) for ci, L in enumerate(lengths) for w in genome.contig_windows(L, win)}
    assert max(loads) - min(loads) <= win and sum(loads) == sum(lengths)
    # configs[4]: window k*step .. k*step + win, contiguous blocks in rank order
    step, win4, L4 = 500, 1000, 200_000_000
    nwin = (L4 - win4) // step + 1
    k = 0
    for r in range(world):
        (seg,), _ = res[r][4]
        ci, b, e, st, lo, hi = seg
        assert st == step and lo == k * step and b == lo and e == (hi // step - 1) * step + win4
        k = hi // step
    assert k == nwin
