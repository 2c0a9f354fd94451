"""Whole-genome pass (BASELINE.json configs[3]: 3 Gbp x 24 samples, 24 contigs of 125 Mbp,
nucdiv + sfs + ld + diverge over 10 kb windows) on one GPU, and its contig-first shard plan
across GPUs.

The reference walks a genome window by window, re-fetching each window's reads through the
BAM index (pop_nucdiv.cpp:45-125), so its memory is O(window).  Here the pileup of a genome
does not fit HBM (3 Gbp x 24 samples x depth 10 is ~1.8 TB of keys) but its packed rows do
(4 bytes per position: 12 GB), so the pass streams the pileup in chunks and keeps the rows:

    for each chunk of each contig (multiple of 64 positions):
        producer stream: pileup chunk -> buffer[c % 2]      (pbg_synth_pileup here; the host
                                                             feeder's H2D copy in a real run)
        call stream:     pbg_call_sites(buffer[c % 2]) -> rows[contig base + chunk offset]
    for each contig: pbg_window_stats(rows of the contig, the contig's windows)

Two pileup buffers alternate; events order producer and consumer, so the generation of chunk
c+1 overlaps the call of chunk c.  A window never straddles contigs and every window reads
only rows, so no halo is carried between chunks: the chunked rows equal the one-batch rows
position for position (tests/test_genome.py).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib, workload

SITE_BLOCK = _lib.PBG_SITE_BLOCK


@dataclass
class Segment:
    """Positions [beg, end) of contig `contig` (0-based), a whole number of windows.  With
    step > 0 the windows are [a, a + win) for a in range(win_lo, win_hi, step) (overlapping
    windows, BASELINE configs[4]; the reference has no step option) and [beg, end) includes
    the halo the last of them reads."""
    contig: int
    beg: int
    end: int
    step: int = 0
    win_lo: int = 0
    win_hi: int = 0


def contig_windows(length: int, win: int, beg: int = 0, end: int | None = None):
    """The reference's window list of [beg, end) of a contig (pop_nucdiv.cpp:49, 63)."""
    return workload.reference_windows(beg, length if end is None else end, win)


def plan_genome(lengths: list[int], world: int, win: int) -> list[list[Segment]]:
    """Contig-first shard plan: whole contigs go to the rank with the fewest
    positions so far (largest first); when there are fewer contigs than ranks, or a contig is
    much larger than a rank's share, it is split at window borders into pieces of about the
    per-rank share.  Every window of every contig lands on exactly one rank, in one piece."""
    total = sum(lengths)
    share = max(win, -(-total // max(1, world)))
    pieces: list[Segment] = []
    for ci, L in enumerate(lengths):
        nw = max(0, (L - 1) // win)
        if L <= share or nw <= 1:
            pieces.append(Segment(ci, 0, L))
            continue
        per = max(1, -(-nw // -(-L // share)))          # windows per piece
        for a in range(0, nw, per):
            b = min(nw, a + per)
            # region whose window loop is windows [a, b) of the contig (popbam_amd.shard geometry)
            pieces.append(Segment(ci, a * win, b * win + 1 if b < nw else L))
    load = [0] * world
    plan: list[list[Segment]] = [[] for _ in range(world)]
    for p in sorted(pieces, key=lambda s: s.end - s.beg, reverse=True):
        r = min(range(world), key=lambda k: load[k])
        plan[r].append(p)
        load[r] += p.end - p.beg
    for r in range(world):
        plan[r].sort(key=lambda s: (s.contig, s.beg))
    return plan


def plan_overlapping(length: int, world: int, win: int, step: int) -> list[list[Segment]]:
    """Overlapping windows [k*step, k*step + win) of one contig split into contiguous blocks of
    windows, one per rank (each shard reads a halo of win - step positions)."""
    nwin = max(0, (length - win) // step + 1)
    plan = []
    for r in range(world):
        q, rem = divmod(nwin, world)
        k0 = r * q + min(r, rem)
        k1 = k0 + q + (1 if r < rem else 0)
        plan.append([Segment(0, k0 * step, (k1 - 1) * step + win, step, k0 * step, k1 * step)] if k1 > k0 else [])
    return plan


def rank_plan(config: int, lengths: list[int], world: int, rank: int, win: int, step: int = 0):
    """A rank's segments and statistics for BASELINE configs[3] (contig-first shards of the
    whole genome: nucdiv + sfs + ld ZnS + diverge) or configs[4] (one contig, overlapping
    windows in contiguous blocks with their halo: nucdiv + sfs + haplo EHHS)."""
    if config == 4:
        return (plan_overlapping(lengths[0], world, win, step)[rank],
                _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_HAP_EHHS)
    return (plan_genome(lengths, world, win)[rank],
            _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS | _lib.PBG_S_DIV_IND)


class GenomePass:
    """Streams the synthetic pileup of `segments` through the call kernels chunk by chunk
    (double-buffered, producer and call on separate streams) into genome-resident rows, then
    runs the window statistics per segment.  One `run()` = one pass over every position."""

    def __init__(self, ctx: _lib.Context, segments: list[Segment], seed: int, mean_depth: int = 10,
                 win: int = 10_000, stats: int = 0, chunk: int = 1 << 25, device: str = "cuda",
                 serial: bool = False):
        assert chunk % SITE_BLOCK == 0
        self.ctx, self.segments, self.seed, self.mean_depth, self.win = ctx, segments, seed, mean_depth, win
        self.stats, self.chunk = stats, chunk
        # serial: each chunk is generated on the call stream right before its call (the call's
        # kernels then have the GPU to themselves); else double-buffered on two streams
        self.serial = serial
        rb = ctx.row_bytes
        # rows: one region per segment, each starting 16-byte aligned
        self.row_base = []
        off = 0
        for s in segments:
            self.row_base.append(off)
            off += ((s.end - s.beg) * rb + 255) // 256 * 256   # 256-byte aligned: whole row indices
        self.rows = torch.zeros(max(off, 256), dtype=torch.uint8, device=device)
        # chunks: (segment index, first position, positions)
        self.chunks = []
        for si, s in enumerate(segments):
            for p in range(s.beg, s.end, chunk):
                self.chunks.append((si, p, min(chunk, s.end - p)))
        n = ctx.params.n_samples
        spec = _lib.PbgSynthSpec(seed, 0, mean_depth, 0, chunk)
        self.keys_cap = int(ctx.lib.pbg_synth_max_keys(ctx.h, C.byref(spec)))
        kt = torch.uint8 if ctx.k_bytes == 1 else torch.int16
        nblk = chunk // SITE_BLOCK
        self.buf = [dict(ref=torch.empty(chunk, dtype=torch.uint8, device=device),
                         k=torch.empty(chunk * n, dtype=kt, device=device),
                         rmsq=torch.empty(chunk * n, dtype=torch.int32, device=device),
                         block_off=torch.zeros(nblk + 1, dtype=torch.int64, device=device),
                         keys=torch.empty(max(8, self.keys_cap), dtype=torch.int16, device=device))
                    for _ in range(1 if serial else 2)]
        self.key_total = torch.zeros(1, dtype=torch.int64, device=device)   # keys called (SURVEY 8(d) bytes)
        self.gen_stream = torch.cuda.Stream(device=device)
        self.call_stream = torch.cuda.Stream(device=device)
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [torch.cuda.Event() for _ in range(2)]
        self.slot_used = [False, False]   # a call on the slot's buffer has been enqueued (free[] recorded)
        # windows of every segment as row indices into the genome-resident rows; one statistics
        # launch per group of segments whose rows stay below 2^31 (pbg_window is int32)
        self.win_lists = []
        self.groups = []   # (first row byte, rows, window list)
        for si, s in enumerate(segments):
            if s.step:
                w = [(a - s.beg, a - s.beg + win) for a in range(s.win_lo, s.win_hi, s.step)]
            else:
                w = [(a - s.beg, b - s.beg) for a, b in contig_windows(s.end, win, s.beg, s.end)]
            self.win_lists.append(w)
            nrows_seg = (s.end - s.beg)
            if not self.groups or (self.row_base[si] - self.groups[-1][0]) // rb + nrows_seg >= (1 << 31) - 256:
                self.groups.append([self.row_base[si], 0, []])
            g = self.groups[-1]
            r0 = (self.row_base[si] - g[0]) // rb
            g[2] += [(r0 + a, r0 + b) for a, b in w]
            g[1] = r0 + nrows_seg
        self.n_windows = sum(len(w) for w in self.win_lists)
        self.gstats = []
        if stats:
            p = ctx.params
            for base, nrows, w in self.groups:
                if not w:
                    continue
                out = workload.WindowOutputs(len(w), p.n_samples, p.n_pops, device, ctx.sfs_stride)
                wins = torch.tensor([x for ab in w for x in ab], dtype=torch.int32).to(device)
                self.gstats.append((base, nrows, wins, len(w), out, out.struct(workload.HotPath.fields_for(stats))))
        self.opts = _lib.PbgStatOpts(stats, 1, 0, 0)

    @property
    def n_sites(self) -> int:
        return sum(s.end - s.beg for s in self.segments)

    def _generate(self, c: int, slot: int, stream=None):
        si, p, L = self.chunks[c]
        s = self.segments[si]
        b = self.buf[slot]
        spec = _lib.PbgSynthSpec(self.seed, s.contig, self.mean_depth, p, L)
        st = (stream or self.gen_stream).cuda_stream
        self.ctx.check(self.ctx.lib.pbg_synth_pileup(self.ctx.h, C.byref(spec), b["ref"].data_ptr(), b["k"].data_ptr(),
                                                     b["rmsq"].data_ptr(), b["block_off"].data_ptr(),
                                                     b["keys"].data_ptr(), self.keys_cap, None, st), "pbg_synth_pileup")

    def _call(self, c: int, slot: int):
        si, p, L = self.chunks[c]
        s = self.segments[si]
        b = self.buf[slot]
        pl = _lib.PbgPileup(L, p, b["ref"].data_ptr(), b["k"].data_ptr(), b["rmsq"].data_ptr(),
                            b["block_off"].data_ptr(), b["keys"].data_ptr())
        rows = self.rows.data_ptr() + self.row_base[si] + (p - s.beg) * self.ctx.row_bytes
        self.ctx.check(self.ctx.lib.pbg_call_sites(self.ctx.h, C.byref(pl), rows, None, self.call_stream.cuda_stream),
                       "pbg_call_sites")

    def call_all(self):
        """Every chunk: generate (producer stream) -> call (call stream), double-buffered; or,
        serial, generate -> call on the call stream."""
        if self.serial:
            for c in range(len(self.chunks)):
                self._generate(c, 0, self.call_stream)
                self._call(c, 0)
                nb = (self.chunks[c][2] + SITE_BLOCK - 1) // SITE_BLOCK
                with torch.cuda.stream(self.call_stream):
                    self.key_total += self.buf[0]["block_off"][nb:nb + 1]
            return
        for c in range(len(self.chunks)):
            slot = c & 1
            with torch.cuda.stream(self.gen_stream):
                # the slot's previous call (this pass or the previous one) must be done with it
                if self.slot_used[slot]:
                    self.gen_stream.wait_event(self.free[slot])
                self.slot_used[slot] = True
                self._generate(c, slot)
                self.ready[slot].record(self.gen_stream)
            with torch.cuda.stream(self.call_stream):
                self.call_stream.wait_event(self.ready[slot])
                self._call(c, slot)
                nb = (self.chunks[c][2] + SITE_BLOCK - 1) // SITE_BLOCK
                self.key_total += self.buf[slot]["block_off"][nb:nb + 1]
                self.free[slot].record(self.call_stream)

    def stats_all(self):
        """pbg_window_stats over every window, one launch per row group, on the call stream."""
        for base, nrows, wins, nw, out, ostruct in self.gstats:
            self.ctx.check(self.ctx.lib.pbg_window_stats(self.ctx.h, self.rows.data_ptr() + base, nrows, wins.data_ptr(), nw,
                                                         C.byref(self.opts), C.byref(ostruct),
                                                         self.call_stream.cuda_stream), "pbg_window_stats")

    def window_results(self, field: str):
        """A pbg_window_out field over all windows (segment order), on the host."""
        import numpy as np
        return np.concatenate([g[4].t[field].cpu().numpy() for g in self.gstats]) if self.gstats else None

    def survey_bytes(self, passes: int = 1) -> int:
        """SURVEY 8(d) call-stage bytes of the positions called so far over `passes` passes:
        2 per key + 5 per (position, sample) + 1 + row_bytes per position."""
        n = self.ctx.params.n_samples
        keys = int(self.key_total.item()) // max(1, passes)
        return 2 * keys + 5 * self.n_sites * n + self.n_sites * (1 + self.ctx.row_bytes)

    def run(self):
        self.call_all()
        if self.stats:
            self.stats_all()

    def synchronize(self):
        self.gen_stream.synchronize()
        self.call_stream.synchronize()
        self.ctx.sync_check(self.call_stream.cuda_stream)

    def segment_rows(self, si: int) -> torch.Tensor:
        s = self.segments[si]
        a = self.row_base[si]
        return self.rows[a:a + (s.end - s.beg) * self.ctx.row_bytes]
