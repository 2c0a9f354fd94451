"""Window-block sharding (popbam_amd.shard): the geometry reproduces the reference's window
list exactly, and a world_size-2 gloo run (one process per rank, no collective on the data
path, text gathered to rank 0) prints what a single run prints.  The per-rank compute here
is the CPU oracle (test infrastructure) so the N>1 path is covered without a GPU; the GPU
variant below runs each rank's block through pbg_run on a sliced, re-based pileup."""
import os
import socket

import numpy as np
import pytest

import fixtures
import harness
from popbam_amd import shard

CASES = [("g01_base", ["nucdiv", "-w", "1"], "chr1"), ("g12_regions", ["sfs", "-w", "2"], "chr1:777-14777"),
         ("g11_eleven", ["ld", "-w", "10"], "chr1"), ("g03_threepops", ["diverge", "-w", "1"], "chr1"),
         ("g12_regions", ["snp"], "chr1:2001-3000"), ("g02_interleaved", ["haplo", "-w", "1", "-o", "2"], "chr1"),
         ("g01_base", ["tree", "-w", "1", "-d", "jc"], "chr1"),
         ("g13_snpformats", ["snp", "-o", "2", "-w", "2"], "chr1"), ("g14_onepop", ["snp", "-o", "2", "-w", "1"], "chr1")]


def _windows(beg, end, w, windowed):
    if not windowed:
        return [(beg, end)]
    return [(beg + cw * w, (cw + 1) * w + beg - 1) for cw in range(shard.num_windows(beg, end, w, True))]


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("beg,end,w", [(0, 30000, 1000), (776, 14777, 2000), (7, 8, 1), (0, 99999, 7),
                                       (100, 50, 10)])
def test_blocks_reproduce_window_list(world, beg, end, w):
    full = _windows(beg, end, w, True)
    got = []
    for r in range(world):
        reg = shard.shard_region(beg, end, w, True, r, world)
        if reg is None:
            continue
        got += _windows(reg[0], reg[1], w, True)
        lo, hi = shard.positions_needed(reg[0], reg[1], w, True)
        sub = _windows(reg[0], reg[1], w, True)
        assert lo == sub[0][0] and hi == sub[-1][1]
    assert got == full
    sizes = [np.subtract(*shard.window_block(len(full), r, world)[::-1]) for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def test_unwindowed_run_goes_to_rank0():
    assert shard.shard_region(5, 900, 0, False, 0, 4) == (5, 900)
    assert all(shard.shard_region(5, 900, 0, False, r, 4) is None for r in range(1, 4))


def test_slice_batch_rebases_reads():
    b = harness.synth_batch(3, 0, 640, 5, 10)
    batch = {"ref": b["ref"], "depth": b["depth"], "reads": b["reads"]}
    sub = shard.slice_batch(batch, 1000, 1100, 1300)
    assert sub["pos0"] == 1100 and len(sub["ref"]) == 200
    ref = harness.synth_batch(3, 100, 300, 5, 10)
    assert np.array_equal(sub["depth"], ref["depth"]) and np.array_equal(sub["reads"], ref["reads"])
    assert len(shard.slice_batch(batch, 0, 700, 900)["ref"]) == 0
    from popbam_amd import workload
    p = workload.default_params(5)
    kb, kref = harness.key_batch(b, p), harness.key_batch(ref, p)
    ksub = shard.slice_batch(kb, 1000, 1100, 1300)
    assert ksub["pos0"] == 1100
    for f in ("ref", "k", "rmsq", "keys"):
        assert np.array_equal(ksub[f], kref[f]), f


def _ms_header(text, ms):
    """The oracle prints a block's own `snp -o 2` header; apply pbg_cmd.ms_windows to it
    (> 0: the run's total window count, < 0: no header)."""
    if not text.startswith("ms ") or ms == 0:
        return text
    head, rest = text.split("\n", 1)
    if ms < 0:
        return rest.split("\n", 2)[2]
    f = head.split(" ")
    f[2] = str(ms)
    return " ".join(f) + "\n" + rest


def _oracle_block(st, b, e, ms=0):
    c0 = (st.beg, st.end)
    st.beg, st.end = b, e
    try:
        return _ms_header(harness.oracle_run(st), ms)
    finally:
        st.beg, st.end = c0


def _worker(rank, world, port, results):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        for i, (name, args, region) in enumerate(CASES):
            st = harness.Setup(name, args, region)
            windowed = bool(st.opts.flag & harness.opt.BAM_WINDOW)
            text = shard.run_sharded(lambda b, e, ms: _oracle_block(st, b, e, ms), st.beg, st.end,
                                     st.opts.win_size, windowed)
            if rank == 0:
                results[i] = text
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_run_matches_single_run(world):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    for i, (name, args, region) in enumerate(CASES):
        st = harness.Setup(name, args, region)
        full = harness.oracle_run(st)
        assert results[i] == full, f"{name} {args}"
        cs = [c for c in fixtures.load_case(name)["meta"]["cases"] if c["args"] == args and c["region"] == region]
        if cs:
            ok, diff = harness.same_output(args, fixtures.golden_text(name, cs[0]["stdout"]), results[i])
            assert ok, diff


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_blocks_on_rebased_pileups(gpu_lib, world):
    """Each rank's block through pbg_run on only the positions it reads (pos0 != 0)."""
    from popbam_amd import engine
    for name, args, region in CASES:
        st = harness.Setup(name, args, region)
        windowed = bool(st.opts.flag & harness.opt.BAM_WINDOW)
        parts = []
        for r in range(world):
            reg = shard.shard_region(st.beg, st.end, st.opts.win_size, windowed, r, world)
            if reg is None:
                continue
            lo, hi = shard.positions_needed(reg[0], reg[1], st.opts.win_size, windowed)
            sub = shard.slice_batch(st.kbatch, 0, lo, max(hi, lo + 1))
            ms = shard.ms_windows_for(st.beg, st.end, st.opts.win_size, windowed, r)
            parts.append(engine.run_command(st.opts, st.sm, st.chr, reg[0], reg[1], sub, pos0=sub["pos0"],
                                            refid=st.refid, ms_windows=ms))
        ours = "".join(parts)
        oob = harness.snp_oob_cells(harness.oracle_run(st)) if args[0] == "snp" else None
        ok, diff = harness.same_output(args, harness.oracle_run(st), ours, oob)
        assert ok, f"{name} {args}: {diff}"
