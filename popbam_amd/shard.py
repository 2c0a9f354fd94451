"""Multi-GPU sharding of one `popbam <cmd>` invocation.

Windows are independent (every statistic of a window reads only that window's rows), so a
run is split into contiguous blocks of windows, one block per rank (one process per GPU),
with no collective on the data path: rank r runs the same window loop as the reference
(pop_nucdiv.cpp:47-124) restricted to its block, and the TSV fragments are concatenated in
rank order.  The only communication is the final gather of the text to rank 0.

Block b of the window list [beg + cw*w, beg + (cw+1)*w - 1), cw in [a, b), is produced
exactly by the reference's own geometry with beg' = beg + a*w and end' = beg + b*w + 1,
since num_windows = ((end' - beg') - 1) / w = b - a and the printed coordinates depend
only on beg + cw*w.  A run without -w is a single window: rank 0 computes it (no
cross-window reduction exists in the reference to split it with).  `snp` prints one line
per segregating position inside each window, so the same split applies.
"""
from __future__ import annotations

import numpy as np


def num_windows(beg: int, end: int, win_size: int, windowed: bool) -> int:
    """Window count of main_<cmd> (pop_nucdiv.cpp:47-48)."""
    if not windowed:
        return 1
    return max(0, ((end - beg) - 1) // win_size)


def window_block(n_win: int, rank: int, world: int) -> tuple[int, int]:
    """Balanced contiguous block [a, b) of n_win windows for `rank` of `world`."""
    q, r = divmod(n_win, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def shard_region(beg: int, end: int, win_size: int, windowed: bool, rank: int, world: int):
    """(beg', end') whose window loop prints exactly this rank's block, or None when the
    rank has no window."""
    if not windowed:
        return (beg, end) if rank == 0 else None
    a, b = window_block(num_windows(beg, end, win_size, True), rank, world)
    if a == b:
        return None
    return beg + a * win_size, beg + b * win_size + 1


def positions_needed(beg: int, end: int, win_size: int, windowed: bool) -> tuple[int, int]:
    """Contig positions [lo, hi) the windows of (beg, end) read (the last base of each
    window is never read, Appendix A.1)."""
    if not windowed:
        return beg, end
    nw = num_windows(beg, end, win_size, True)
    return beg, beg + nw * win_size - 1 if nw else beg


def slice_batch(batch: dict, pos0: int, lo: int, hi: int) -> dict:
    """The part of a host pileup batch (positions [pos0, pos0 + len(ref))) that covers
    [lo, hi): per-position rows and the matching run of reads (raw batch: 'depth' / 'reads')
    or keys (key batch: 'k' / 'rmsq' / 'keys')."""
    n_sites = len(batch["ref"])
    a = min(max(lo - pos0, 0), n_sites)
    b = min(max(hi - pos0, a), n_sites)
    if "keys" in batch:
        k = np.asarray(batch["k"])
        cum = np.concatenate([[0], np.cumsum(k.sum(axis=1, dtype=np.int64))])
        return {"ref": np.asarray(batch["ref"])[a:b], "k": k[a:b], "rmsq": np.asarray(batch["rmsq"])[a:b],
                "keys": np.asarray(batch["keys"])[cum[a]:cum[b]], "pos0": pos0 + a}
    dep = np.asarray(batch["depth"])
    cum = np.concatenate([[0], np.cumsum(dep.sum(axis=1, dtype=np.int64))])
    return {"ref": np.asarray(batch["ref"])[a:b], "depth": dep[a:b],
            "reads": np.asarray(batch["reads"])[cum[a]:cum[b]], "pos0": pos0 + a}


def ms_windows_for(beg: int, end: int, win_size: int, windowed: bool, rank: int) -> int:
    """`snp -o 2` header control for this rank's block (pbg_cmd.ms_windows): the reference
    prints one header, with the whole run's window count, before window 0 (pop_snp.cpp:114-115),
    so rank 0 prints it with the total and every later block prints none."""
    return num_windows(beg, end, win_size, windowed) if rank == 0 else -1


def run_sharded(run_block, beg: int, end: int, win_size: int, windowed: bool, group=None) -> str | None:
    """Run this rank's block with run_block(beg', end', ms_windows) -> str and gather the
    fragments to rank 0 in rank order (returns the full text on rank 0, None elsewhere).
    Without an initialised process group this is a single-rank run."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return run_block(beg, end, 0)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    reg = shard_region(beg, end, win_size, windowed, rank, world)
    text = run_block(*reg, ms_windows_for(beg, end, win_size, windowed, rank)) if reg is not None else ""
    parts = [None] * world if rank == 0 else None
    dist.gather_object(text, parts, dst=0, group=group)
    return "".join(parts) if rank == 0 else None
