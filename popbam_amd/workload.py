"""HBM-resident synthetic workload + the device-side hot path (benchmark / scale tests).

`SynthPileup` generates the counter-based synthetic pileup (splitmix64 keyed
on (seed, position); depth ~ Binomial(2D, 1/2), baseQ 20..40, mapQ 60, ~0.8% errors,
theta ~ 1.2% segregating) straight into device memory with the library's generator kernels.
`HotPath` runs one step -- call kernel + window-statistics kernel -- on it.  torch is used
only to own device memory and streams; all compute is in libpopbam_gpu.so.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

SITE_BLOCK = _lib.PBG_SITE_BLOCK


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def stream_handle(stream: torch.cuda.Stream | None = None) -> int:
    s = stream or torch.cuda.current_stream()
    return s.cuda_stream


def default_params(n_samples: int, n_pops: int = 2, **kw) -> _lib.PbgParams:
    """Contiguous equal populations, reference default filters."""
    p = _lib.PbgParams()
    p.n_samples, p.n_pops = n_samples, n_pops
    per = n_samples // n_pops
    masks = [0] * n_pops
    for i in range(n_samples):
        pi = min(i // per, n_pops - 1)
        masks[pi] |= 1 << i
        p.pop_n[pi] += 1
    for pi, m in enumerate(masks):
        p.set_pop_mask(pi, m)
    p.min_depth, p.max_depth, p.min_rmsQ, p.min_snpQ = 3, 255, 25, 25
    p.min_mapQ, p.min_baseQ, p.flag = 13, 13, 0
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class SynthPileup:
    """Synthetic key batch in HBM (pbg_synth_pileup): positions [pos0, pos0 + n_sites) of
    `contig`, with the context's filters applied.  keys[] is sized exactly (one host sync)
    unless `keys_cap` is given (then no sync: pipelined producers pass the upper bound)."""

    def __init__(self, ctx: _lib.Context, n_sites: int, mean_depth: int = 10, seed: int = 0xC0FFEE02,
                 device: str = "cuda", contig: int = 0, pos0: int = 0, keys_cap: int | None = None,
                 stream: torch.cuda.Stream | None = None):
        self.ctx, self.n_sites, self.mean_depth, self.seed = ctx, n_sites, mean_depth, seed
        self.contig, self.pos0 = contig, pos0
        n = ctx.params.n_samples
        nblk = (n_sites + SITE_BLOCK - 1) // SITE_BLOCK
        self.spec = _lib.PbgSynthSpec(seed, contig, mean_depth, pos0, n_sites)
        self.ref = torch.empty(max(1, n_sites), dtype=torch.uint8, device=device)
        self.k = torch.empty(max(1, n_sites * n), dtype=torch.uint8 if ctx.k_bytes == 1 else torch.int16,
                             device=device)
        self.rmsq = torch.empty(max(1, n_sites * n), dtype=torch.int32, device=device)
        self.block_off = torch.zeros(nblk + 1, dtype=torch.int64, device=device)
        self.max_keys = int(ctx.lib.pbg_synth_max_keys(ctx.h, C.byref(self.spec)))
        if keys_cap is None:   # exact size: a counting pass (keys = NULL), then the batch
            nk = C.c_uint64(0)
            ctx.check(ctx.lib.pbg_synth_pileup(ctx.h, C.byref(self.spec), _ptr(self.ref), _ptr(self.k),
                                               _ptr(self.rmsq), _ptr(self.block_off), None, 0, C.byref(nk),
                                               stream_handle(stream)), "pbg_synth_pileup")
            keys_cap = nk.value
        self.keys_cap = keys_cap
        self.keys = torch.empty(max(8, keys_cap), dtype=torch.int16, device=device)
        self.n_keys = None
        self.generate(stream, sync=True)

    def generate(self, stream=None, sync: bool = True):
        """(Re)generate the batch on `stream` (asynchronous unless sync)."""
        s = stream_handle(stream)
        nk = C.c_uint64(0)
        self.ctx.check(self.ctx.lib.pbg_synth_pileup(self.ctx.h, C.byref(self.spec), _ptr(self.ref), _ptr(self.k),
                                                     _ptr(self.rmsq), _ptr(self.block_off), _ptr(self.keys),
                                                     self.keys_cap, C.byref(nk) if sync else None, s),
                       "pbg_synth_pileup")
        if sync:
            self.n_keys = nk.value

    def pileup(self) -> _lib.PbgPileup:
        return _lib.PbgPileup(self.n_sites, self.pos0, _ptr(self.ref), _ptr(self.k), _ptr(self.rmsq),
                              _ptr(self.block_off), _ptr(self.keys))

    def survey_bytes(self) -> int:
        """SURVEY 8(d) algorithmic bytes of the call stage for this batch: per (position,
        sample) 2k + 5 (u16 keys, u8 k, u32 sum mapQ^2), per position 1 (reference byte) +
        row_bytes written."""
        n = self.ctx.params.n_samples
        return 2 * self.n_keys + 5 * self.n_sites * n + self.n_sites * (1 + self.ctx.row_bytes)

    def layout_bytes_scan(self) -> int:
        """Bytes one call_scan_kernel launch must move in this layout: the keys, k (k_bytes),
        rmsq, reference bytes and block offsets read, one info byte per (position, sample)
        written (queue entries not counted)."""
        n = self.ctx.params.n_samples
        nblk = (self.n_sites + SITE_BLOCK - 1) // SITE_BLOCK
        return (2 * self.n_keys + (self.ctx.k_bytes + 4 + 1) * self.n_sites * n + self.n_sites +
                8 * (nblk + 1))


def reference_windows(beg: int, end: int, win_size: int):
    """main_<cmd> window list (pop_nucdiv.cpp:49, 63): [beg+cw*w, beg+(cw+1)*w-1)."""
    nw = ((end - beg) - 1) // win_size
    return [(beg + cw * win_size, (cw + 1) * win_size + beg - 1) for cw in range(nw)]


class WindowOutputs:
    """Device arrays for pbg_window_out (all statistics)."""

    def __init__(self, n_win: int, n: int, np_: int, device: str = "cuda", sfs_stride: int | None = None):
        npairs = max(1, np_ * (np_ - 1))
        sfs_stride = sfs_stride or n + 1
        f64 = dict(dtype=torch.float64, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        self.t = {
            "num_sites": torch.zeros(n_win, **i32), "segsites": torch.zeros(n_win, **i32),
            "pi": torch.zeros(n_win * np_, **f64), "dxy": torch.zeros(n_win * npairs, **f64),
            "td": torch.zeros(n_win * np_, **f64), "fwh": torch.zeros(n_win * np_, **f64),
            "ld_snps": torch.zeros(n_win * np_, **i32), "ld_val": torch.zeros(n_win * np_, **f64),
            "ld_q": torch.zeros(n_win * np_, **f64), "div_ind": torch.zeros(n_win * n, **f64),
            "div_fixed": torch.zeros(n_win * np_, **i32), "div_seg": torch.zeros(n_win * np_, **i32),
            "div_pop": torch.zeros(n_win * np_, **f64), "nhaps": torch.zeros(n_win * np_, **i32),
            "hap_val": torch.zeros(n_win * np_, **f64), "hap_dxy": torch.zeros(n_win * npairs, **f64),
            "hap_min": torch.zeros(n_win * npairs, **i32),
            "tree_diff": torch.zeros(n_win * (n + 1) * (n + 1), **i32),
            "sfs_bins": torch.zeros(n_win * np_ * sfs_stride, **i32), "seg_pop": torch.zeros(n_win * np_, **i32),
            "theta_w": torch.zeros(n_win * np_, **f64),
        }

    def struct(self, fields) -> _lib.PbgWindowOut:
        o = _lib.PbgWindowOut()
        for k in fields:
            setattr(o, k, _ptr(self.t[k]))
        return o


class HotPath:
    """call kernel (pileup -> rows) + window-statistics kernel (rows -> per-window stats)."""

    def __init__(self, ctx: _lib.Context, synth: SynthPileup, windows, stats: int, min_freq: int = 1,
                 device: str = "cuda"):
        self.ctx, self.synth, self.stats = ctx, synth, stats
        self.rows = torch.zeros(synth.n_sites * ctx.row_bytes, dtype=torch.uint8, device=device)
        self.windows = [tuple(ab) for ab in windows]
        w = torch.tensor([x for ab in windows for x in ab], dtype=torch.int32)
        self.wins = w.to(device)
        self.n_win = len(windows)
        p = ctx.params
        self.out = WindowOutputs(self.n_win, p.n_samples, p.n_pops, device, ctx.sfs_stride)
        fields = self.fields_for(stats)
        self.out_struct = self.out.struct(fields)
        self.opts = _lib.PbgStatOpts(stats, min_freq, 0, 0)
        self.pl = synth.pileup()

    @staticmethod
    def fields_for(stats: int) -> list[str]:
        """pbg_window_out fields a statistics mask writes."""
        fields = ["num_sites", "segsites"]
        if stats & _lib.PBG_S_NUCDIV:
            fields += ["pi", "dxy"]
        if stats & _lib.PBG_S_SFS:
            fields += ["td", "fwh", "sfs_bins", "seg_pop", "theta_w"]
        if stats & (_lib.PBG_S_ZNS | _lib.PBG_S_OMEGA | _lib.PBG_S_WALL):
            fields += ["ld_snps", "ld_val", "ld_q"]
        if stats & _lib.PBG_S_DIV_IND:
            fields += ["div_ind"]
        if stats & _lib.PBG_S_DIV_POP:
            fields += ["div_fixed", "div_seg", "div_pop"]
        if stats & (_lib.PBG_S_HAP_K | _lib.PBG_S_HAP_EHHS | _lib.PBG_S_HAP_DXY):
            fields += ["nhaps", "hap_val", "hap_dxy", "hap_min"]
        if stats & _lib.PBG_S_TREE:
            fields += ["tree_diff"]
        return fields

    def to_host(self) -> dict:
        """The batch's arrays copied once into pinned host memory (the host side of the drop-in
        boundary: what the feeder hands over)."""
        n_keys = int(self.synth.block_off[-1].item())
        s = self.synth
        h = {}
        for name, t in (("ref", s.ref), ("k", s.k), ("rmsq", s.rmsq), ("block_off", s.block_off),
                        ("keys", s.keys[:max(8, n_keys)])):
            h[name] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h[name].copy_(t)
        return h

    def call(self, stream=None, cb: torch.Tensor | None = None):
        s = stream_handle(stream)
        self.ctx.check(self.ctx.lib.pbg_call_sites(self.ctx.h, C.byref(self.pl), _ptr(self.rows),
                                                   _ptr(cb) if cb is not None else None, s), "pbg_call_sites")

    def window_stats(self, stream=None):
        s = stream_handle(stream)
        self.ctx.check(self.ctx.lib.pbg_window_stats(self.ctx.h, _ptr(self.rows), self.synth.n_sites, _ptr(self.wins),
                                                     self.n_win, C.byref(self.opts), C.byref(self.out_struct), s),
                       "pbg_window_stats")

    def step(self, stream=None):
        self.call(stream)
        self.window_stats(stream)

    # ---- pipelined step: the contig in pieces, statistics of piece i beside the call of i+1
    def split_points(self, pieces: int) -> list[int]:
        """Row positions [0, p1, ..., n_sites) splitting the batch into about `pieces` equal
        parts, each split a multiple of the 64-position block with no window across it (so
        every window's rows come from one piece's call)."""
        import bisect
        n = self.synth.n_sites
        wins = sorted(self.windows)
        begs = [b for b, _ in wins]
        reach, m = [], 0   # reach[i] = max end of wins[:i+1]
        for _, e in wins:
            m = max(m, e)
            reach.append(m)

        def free(p):   # no window with beg < p < end
            i = bisect.bisect_left(begs, p)   # wins[:i] begin before p
            return i == 0 or reach[i - 1] <= p

        pts = [0]
        for j in range(1, pieces):
            p = (n * j // pieces) // SITE_BLOCK * SITE_BLOCK
            while p > pts[-1] and not free(p):
                p -= SITE_BLOCK
            if p > pts[-1]:
                pts.append(p)
        pts.append(n)
        return pts

    def pipeline(self, pieces: int, device: str = "cuda"):
        """Per-piece sub-batches (views into the synthetic batch: block_off keeps absolute key
        offsets, so keys[] is shared), row slices, window lists and output slices."""
        n = self.ctx.params.n_samples
        rb, kb = self.ctx.row_bytes, self.ctx.k_bytes
        pts = self.split_points(pieces)
        s = self.synth
        per_win = {k: (t.numel() // max(1, self.n_win), t.element_size()) for k, t in self.out.t.items()}
        fields = self.fields_for(self.stats)
        self.pieces = []
        for p0, p1 in zip(pts[:-1], pts[1:]):
            pl = _lib.PbgPileup(p1 - p0, s.pos0 + p0, _ptr(s.ref) + p0, _ptr(s.k) + p0 * n * kb,
                                _ptr(s.rmsq) + p0 * n * 4, _ptr(s.block_off) + (p0 // SITE_BLOCK) * 8, _ptr(s.keys))
            idx = [i for i, (b, e) in enumerate(self.windows) if b >= p0 and e <= p1]
            assert idx == list(range(idx[0], idx[-1] + 1)) if idx else True
            w = torch.tensor([x for i in idx for x in (self.windows[i][0] - p0, self.windows[i][1] - p0)],
                             dtype=torch.int32).to(device)
            o = _lib.PbgWindowOut()
            w0 = idx[0] if idx else 0
            for k in fields:
                per, es = per_win[k]
                setattr(o, k, _ptr(self.out.t[k]) + w0 * per * es)
            self.pieces.append((pl, _ptr(self.rows) + p0 * rb, p1 - p0, w, len(idx), o))
        assert sum(pc[4] for pc in self.pieces) == self.n_win, "a window spans a piece border"
        self.ev_done = [torch.cuda.Event() for _ in self.pieces]    # piece's call enqueued
        self.ev_stats = [torch.cuda.Event() for _ in self.pieces]   # piece's statistics enqueued
        return pts

    def call_pieces(self, stream):
        for pl, rows, _, _, _, _ in self.pieces:
            self.ctx.check(self.ctx.lib.pbg_call_sites(self.ctx.h, C.byref(pl), rows, None, stream.cuda_stream),
                           "pbg_call_sites")

    def stats_pieces(self, stream):
        for _, rows, nrows, w, nw, o in self.pieces:
            if nw:
                self.ctx.check(self.ctx.lib.pbg_window_stats(self.ctx.h, rows, nrows, _ptr(w), nw, C.byref(self.opts),
                                                             C.byref(o), stream.cuda_stream), "pbg_window_stats")

    def step_pipelined(self, call_stream, stats_stream):
        """call(piece i) on call_stream; stats(piece i) on stats_stream after it.  The statistics
        of piece i run beside the call of piece i+1, and the last piece's beside the next step's
        first call; a piece's call waits only for the previous statistics of that same piece
        (the one reader of its rows).  Same work as step(); the caller synchronises both
        streams before reading outputs."""
        lib, h = self.ctx.lib, self.ctx.h
        for (pl, rows, nrows, w, nw, o), ev, done in zip(self.pieces, self.ev_done, self.ev_stats):
            call_stream.wait_event(done)   # no-op until the piece's statistics have been enqueued once
            self.ctx.check(lib.pbg_call_sites(h, C.byref(pl), rows, None, call_stream.cuda_stream), "pbg_call_sites")
            ev.record(call_stream)
            stats_stream.wait_event(ev)
            if nw:
                self.ctx.check(lib.pbg_window_stats(h, rows, nrows, _ptr(w), nw, C.byref(self.opts), C.byref(o),
                                                    stats_stream.cuda_stream), "pbg_window_stats")
            done.record(stats_stream)
        for (pl, rows, nrows, w, nw, o), ev in zip(self.pieces, self.ev_done):
            self.ctx.check(lib.pbg_call_sites(h, C.byref(pl), rows, None, call_stream.cuda_stream), "pbg_call_sites")
            ev.record(call_stream)
            stats_stream.wait_event(ev)
            if nw:
                self.ctx.check(lib.pbg_window_stats(h, rows, nrows, _ptr(w), nw, C.byref(self.opts), C.byref(o),
                                                    stats_stream.cuda_stream), "pbg_window_stats")
        call_stream.wait_stream(stats_stream)
