"""One `popbam <cmd>` invocation on the GPU (host-side mirror of main_<cmd>).

`run_command` takes what the reference derives before its window loop -- parsed options
(popbam_amd.options), the @RG sample model, the region -- plus the key batch the host side
of the pileup callback produced (popbam_amd.feed: pileup, per-sample partition and call_base's
per-read loop), and returns the reference's stdout.  All compute runs in libpopbam_gpu.so
(pbg_run); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from . import feed
from . import options as opt


def max_depth_of(o: opt.Options) -> int:
    """-x as call_base applies it (popbam.cpp:209-246): the first max_depth reads of a sample
    are kept, so 0 keeps none (every sample fails qfilter's depth test unless -m 0).  The
    pileup holds at most 8000 reads per position (bam_pileup.c:375), so every -x above 65535
    (the k width the device stores) behaves like 65535.  A negative -x makes the reference's
    read buffer allocation throw (new[] of a negative size); it is refused here instead."""
    if o.max_depth < 0:
        raise opt.PopbamError(f"maximum read depth -x {o.max_depth} must not be negative")
    return min(o.max_depth, 65535)


def make_params(o: opt.Options, sm: opt.SampleModel) -> _lib.PbgParams:
    masks, counts = sm.pop_masks()
    if len(masks) > _lib.PBG_MAX_POPS:
        raise opt.PopbamError(f"more than {_lib.PBG_MAX_POPS} populations")
    if sm.n > _lib.PBG_MAX_SAMPLES:
        raise opt.PopbamError(f"more than {_lib.PBG_MAX_SAMPLES} samples")
    p = _lib.PbgParams()
    p.n_samples, p.n_pops = sm.n, len(masks)
    for i, (m, c) in enumerate(zip(masks, counts)):
        p.set_pop_mask(i, m)
        p.pop_n[i] = c
    p.min_depth, p.max_depth = o.min_depth, max_depth_of(o)
    p.min_rmsQ, p.min_snpQ = o.min_rmsQ, o.min_snpQ
    p.min_mapQ, p.min_baseQ = o.min_mapQ & 0xFF, o.min_baseQ & 0xFF
    p.flag = o.flag
    return p


def make_filter(o: opt.Options):
    """call_base's per-read filters for the host side of the callback (popbam.cpp:266-281)."""
    return feed.make_filter(o.min_baseQ, o.min_mapQ, o.flag, max_depth_of(o))


class _Cmd:
    def __init__(self, o: opt.Options, sm: opt.SampleModel, chr_name: str, beg: int, end: int,
                 refid: str = "", ms_windows: int = 0):
        c = _lib.PbgCmd()
        c.cmd = opt.CMD_IDS[o.cmd]
        c.output, c.min_sites, c.min_snps, c.min_freq = o.output, o.min_sites, o.min_snps, o.min_freq
        c.outidx = 0
        if o.flag & opt.BAM_OUTGROUP and o.cmd in ("sfs", "diverge", "snp"):   # nucdiv sets the flag, never reads -p
            idx = [i for i, s in enumerate(sm.samples) if s == o.outgroup]
            if not idx:
                raise opt.PopbamError(f"Specified outgroup {o.outgroup} not found")
            c.outidx = idx[-1]
        c.jc = 1 if o.dist == "jc" else 0
        c.windowed = 1 if o.flag & opt.BAM_WINDOW else 0
        c.win_size = o.win_size
        c.beg, c.end = beg, end
        self._chr = chr_name.encode()
        self._sn = (C.c_char_p * max(1, sm.n))(*[s.encode() for s in sm.samples])
        self._pn = (C.c_char_p * max(1, len(sm.pops)))(*[p.encode() for p in sm.pops])
        c.chr_name = self._chr
        c.sample_names = C.cast(self._sn, C.POINTER(C.c_char_p))
        c.pop_names = C.cast(self._pn, C.POINTER(C.c_char_p))
        self._refid = refid.encode()
        c.refid = self._refid
        c.ms_windows = ms_windows
        self.c = c


def run_command(o: opt.Options, sm: opt.SampleModel, chr_name: str, beg: int, end: int, batch: dict,
                pos0: int = 0, device: int = 0, ctx: _lib.Context | None = None, refid: str = "",
                ms_windows: int = 0) -> str:
    """batch: the key batch {'ref': u8[n_sites], 'k': u8/u16[n_sites, n], 'rmsq': u32[n_sites, n],
    'keys': u16[...]} (host; popbam_amd.feed)."""
    own = ctx is None
    if own:
        ctx = _lib.Context(make_params(o, sm), device)
    try:
        kt = np.uint8 if ctx.k_bytes == 1 else np.uint16
        ref = np.ascontiguousarray(batch["ref"], dtype=np.uint8)
        k = np.ascontiguousarray(batch["k"], dtype=kt)
        rq = np.ascontiguousarray(batch["rmsq"], dtype=np.uint32)
        keys = np.ascontiguousarray(batch["keys"], dtype=np.uint16)
        if keys.size == 0:
            keys = np.zeros(8, np.uint16)
        pl = _lib.PbgPileup(len(ref), pos0, ref.ctypes.data, k.ctypes.data, rq.ctypes.data, None, keys.ctypes.data)
        cmd = _Cmd(o, sm, chr_name, beg, end, refid, ms_windows)
        need = C.c_size_t(0)
        cap = 1 << 20
        buf = C.create_string_buffer(cap)
        r = ctx.lib.pbg_run(ctx.h, C.byref(cmd.c), C.byref(pl), buf, cap, C.byref(need))
        if r == _lib.PBG_E_RANGE and need.value > cap:
            buf = C.create_string_buffer(need.value)   # the text is kept by the context
            r = ctx.lib.pbg_take_text(ctx.h, buf, need.value)
        ctx.check(r, "pbg_run")
        return buf.value.decode()
    finally:
        if own:
            ctx.close()


def run_command_sharded(o: opt.Options, sm: opt.SampleModel, chr_name: str, beg: int, end: int, batch: dict,
                        pos0: int = 0, device: int = 0, group=None, refid: str = "") -> str | None:
    """run_command over this rank's block of windows (popbam_amd.shard), on this rank's GPU,
    with the TSV gathered to rank 0.  Each rank uploads only the positions its windows read."""
    from . import shard
    windowed = bool(o.flag & opt.BAM_WINDOW)

    def block(b, e, ms):
        lo, hi = shard.positions_needed(b, e, o.win_size, windowed)
        hi = max(hi, lo + 1)
        sub = shard.slice_batch(batch, pos0, lo, hi)
        return run_command(o, sm, chr_name, b, e, sub, pos0=sub["pos0"], device=device, refid=refid,
                           ms_windows=ms)

    return shard.run_sharded(block, beg, end, o.win_size, windowed, group)
