"""Shared test harness: option/region/sample setup for a golden case, plus the ctypes
binding of the CPU oracle (oracle/liboracle.so -- test infrastructure, the checker)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from popbam_amd import options as opt  # noqa: E402
import fixtures  # noqa: E402

ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")


class OrcParams(C.Structure):
    _fields_ = [("n_samples", C.c_int32), ("n_pops", C.c_int32), ("pop_mask", C.c_uint64 * 64),
                ("pop_n", C.c_int32 * 64), ("min_depth", C.c_int32), ("max_depth", C.c_int32),
                ("min_rmsQ", C.c_int32), ("min_snpQ", C.c_int32), ("min_mapQ", C.c_int32),
                ("min_baseQ", C.c_int32), ("flag", C.c_uint32), ("pop_mask_hi", C.c_uint64 * 64)]


class OrcCmd(C.Structure):
    _fields_ = [("cmd", C.c_int32), ("output", C.c_int32), ("min_sites", C.c_int32), ("min_snps", C.c_int32),
                ("min_freq", C.c_int32), ("outidx", C.c_int32), ("jc", C.c_int32), ("windowed", C.c_int32),
                ("win_size", C.c_int64), ("beg", C.c_int32), ("end", C.c_int32), ("chr_name", C.c_char_p),
                ("sample_names", C.POINTER(C.c_char_p)), ("pop_names", C.POINTER(C.c_char_p)),
                ("refid", C.c_char_p)]


_orc = None


def oracle():
    global _orc
    if _orc is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True,
                           capture_output=True)
        lib = C.CDLL(ORACLE_SO)
        P = C.POINTER
        lib.orc_run.restype = C.c_long
        lib.orc_run.argtypes = [P(OrcParams), P(OrcCmd), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_char_p, C.c_size_t]
        lib.orc_call_sites.restype = C.c_int
        lib.orc_call_sites.argtypes = [P(OrcParams), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.orc_windows_from_sites.restype = C.c_long
        lib.orc_windows_from_sites.argtypes = [P(OrcParams), P(OrcCmd), C.c_void_p, C.c_void_p, C.c_uint32,
                                               C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t]
        lib.orc_sfs_windows.restype = C.c_long
        lib.orc_sfs_windows.argtypes = [P(OrcParams), P(OrcCmd), C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                        C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.orc_synth_batch.restype = C.c_uint64
        lib.orc_synth_batch.argtypes = [C.c_uint64, C.c_int32, C.c_uint64, C.c_uint32, C.c_int32, C.c_int32,
                                        C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        for nm in ("orc_fk", "orc_beta", "orc_lhet"):
            getattr(lib, nm).restype = P(C.c_double)
        _orc = lib
    return _orc


class Setup:
    """Everything a run of `popbam <cmd> ... in.bam <region>` needs, derived exactly as the
    reference derives it."""

    def __init__(self, case_name, args, region):
        self.case = fixtures.load_case(case_name)
        self.opts = opt.parse_args(args[0], list(args[1:]) + ["in.bam", region])
        o = self.opts
        names = [r[0] for r in self.case["refs"]]
        lens = [r[1] for r in self.case["refs"]]
        self.tid, self.beg, self.end = opt.parse_region(o.region, names, lens)
        self.sm = opt.parse_header(self.case["header"], "in.bam")
        self.masks, self.pop_n = self.sm.pop_masks()
        self.outidx = 0
        if o.flag & opt.BAM_OUTGROUP:
            self.outidx = max(i for i, s in enumerate(self.sm.samples) if s == o.outgroup)
        self.chr = names[self.tid]
        self.refid = opt.get_refid(self.case["header"]) if args[0] == "tree" else ""
        self.batch = fixtures.case_batch(case_name, o.max_depth)
        self._kbatch = None

    @property
    def kbatch(self):
        """The fixture's key batch (feed.pack of the raw batch with this command's filters)."""
        if self._kbatch is None:
            from popbam_amd import engine, feed
            self._kbatch = feed.pack(self.batch, self.sm.n, engine.make_filter(self.opts))
        return self._kbatch

    def orc_params(self):
        o = self.opts
        p = OrcParams()
        p.n_samples, p.n_pops = self.sm.n, len(self.sm.pops)
        for i, (m, c) in enumerate(zip(self.masks, self.pop_n)):
            p.pop_mask[i], p.pop_mask_hi[i], p.pop_n[i] = m & ((1 << 64) - 1), m >> 64, c
        p.min_depth, p.max_depth, p.min_rmsQ, p.min_snpQ = o.min_depth, o.max_depth, o.min_rmsQ, o.min_snpQ
        p.min_mapQ, p.min_baseQ, p.flag = o.min_mapQ & 0xFF, o.min_baseQ & 0xFF, o.flag
        return p

    def orc_cmd(self):
        o = self.opts
        c = OrcCmd()
        c.cmd = opt.CMD_IDS[o.cmd]
        c.output = o.output
        c.min_sites = o.min_sites
        c.min_snps = o.min_snps
        c.min_freq = o.min_freq
        c.outidx = self.outidx
        c.jc = 1 if o.dist == "jc" else 0
        c.windowed = 1 if o.flag & opt.BAM_WINDOW else 0
        c.win_size = o.win_size
        c.beg, c.end = self.beg, self.end
        self._keep = [self.chr.encode()] + [s.encode() for s in self.sm.samples] + [p.encode() for p in self.sm.pops]
        c.chr_name = self._keep[0]
        sn = (C.c_char_p * max(1, self.sm.n))(*[s.encode() for s in self.sm.samples])
        pn = (C.c_char_p * max(1, len(self.sm.pops)))(*[p.encode() for p in self.sm.pops])
        self._arrs = (sn, pn)
        c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
        c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
        self._refid = self.refid.encode()
        c.refid = self._refid
        return c


def oracle_run(setup: Setup) -> str:
    lib = oracle()
    b = setup.batch
    p, c = setup.orc_params(), setup.orc_cmd()
    ref = np.ascontiguousarray(b["ref"])
    dep = np.ascontiguousarray(b["depth"])
    rd = np.ascontiguousarray(b["reads"]) if len(b["reads"]) else np.zeros(1, np.uint32)
    cap = 1 << 20
    while True:
        buf = C.create_string_buffer(cap)
        r = lib.orc_run(C.byref(p), C.byref(c), len(ref), ref.ctypes.data, dep.ctypes.data, rd.ctypes.data, buf, cap)
        if r >= 0:
            return buf.value.decode()
        if r == -1:
            raise RuntimeError("orc_run failed")
        cap = -r + 16


def all_cases():
    out = []
    for name in fixtures.case_dirs():
        meta = fixtures.load_case(name)["meta"]
        for i, cs in enumerate(meta["cases"]):
            out.append((name, i))
    return out


def same_output(args, golden: str, ours: str, oob_cells=None):
    """Exact text equality, except snp -o 0 base cells where the reference read iupac[]
    out of bounds (undefined behaviour): the oracle prints '?' there, and for other outputs
    the cells the oracle marked (`oob_cells`) match anything.
    Returns (ok, first differing (golden, ours) line pair)."""
    if args[0] != "snp":
        if golden == ours:
            return True, None
    gl, ol = golden.splitlines(), ours.splitlines()
    if len(gl) != len(ol):
        return False, (f"{len(gl)} lines", f"{len(ol)} lines")
    oob_ok = args[0] == "snp"
    oob_cells = oob_cells or set()
    for li, (a, b) in enumerate(zip(gl, ol)):
        if a == b:
            continue
        fa, fb = a.split("\t"), b.split("\t")
        if oob_ok and len(fa) == len(fb) and all(
                x == y or y == "?" or (li, j) in oob_cells for j, (x, y) in enumerate(zip(fa, fb))):
            continue
        return False, (a, b)
    return True, None


def snp_oob_cells(oracle_text: str):
    """(line, column) of cells the oracle marked '?' (reference UB)."""
    out = set()
    for i, line in enumerate(oracle_text.splitlines()):
        for j, f in enumerate(line.split("\t")):
            if f == "?":
                out.add((i, j))
    return out


def synth_batch(seed, pos_lo, pos_hi, n, mean_depth, max_depth=255, contig=0):
    """Regenerate positions [pos_lo, pos_hi) of the synthetic pileup on the CPU (oracle copy
    of the generator) as a raw host batch (the callback's partition, max_depth cap applied)."""
    lib = oracle()
    L = pos_hi - pos_lo
    ref = np.zeros(max(L, 1), np.uint8)
    dep = np.zeros((max(L, 1), n), np.uint16)
    reads = np.zeros(max(1, L * n * min(2 * mean_depth, max_depth)), np.uint32)
    nr = lib.orc_synth_batch(seed, contig, pos_lo, L, n, mean_depth, max_depth, ref.ctypes.data, dep.ctypes.data,
                             reads.ctypes.data)
    return dict(ref=ref[:L], depth=dep[:L], reads=reads[:nr].copy())


def key_batch(batch, params):
    """The key batch the host side of the callback builds from a raw batch (product code:
    libpopbam_feed.so pbf_pack, call_base's per-read loop) -- what the GPU is given."""
    from popbam_amd import feed
    flt = feed.make_filter(params.min_baseQ, params.min_mapQ, params.flag, params.max_depth)
    return feed.pack(batch, params.n_samples, flt)


def oracle_params_from(pbg_params):
    p = OrcParams()
    p.n_samples, p.n_pops = pbg_params.n_samples, pbg_params.n_pops
    for i in range(pbg_params.n_pops):
        p.pop_mask[i], p.pop_mask_hi[i] = pbg_params.pop_mask[i], pbg_params.pop_mask_hi[i]
        p.pop_n[i] = pbg_params.pop_n[i]
    p.min_depth, p.max_depth = pbg_params.min_depth, pbg_params.max_depth
    p.min_rmsQ, p.min_snpQ = pbg_params.min_rmsQ, pbg_params.min_snpQ
    p.min_mapQ, p.min_baseQ, p.flag = pbg_params.min_mapQ, pbg_params.min_baseQ, pbg_params.flag
    return p


def oracle_call(p, batch):
    """orc_call_sites over a host batch -> (cb[L,n], types, fq[L], flags[L]); types is [L] u64
    for n <= 64, [L, 2] (low, high word) beyond."""
    lib = oracle()
    L, n = batch["depth"].shape
    cb = np.zeros((L, n), np.uint64)
    types = np.zeros(L, np.uint64) if n <= 64 else np.zeros((L, 2), np.uint64)
    fq = np.zeros(L, np.int16)
    flags = np.zeros(L, np.uint8)
    rd = np.ascontiguousarray(batch["reads"] if len(batch["reads"]) else np.zeros(1, np.uint32))
    ref, dep = np.ascontiguousarray(batch["ref"]), np.ascontiguousarray(batch["depth"])   # alive across the call
    assert lib.orc_call_sites(C.byref(p), L, ref.ctypes.data, dep.ctypes.data, rd.ctypes.data,
                              cb.ctypes.data, types.ctypes.data, fq.ctypes.data, flags.ctypes.data) == 0
    return cb, types, fq, flags


def rows_from_oracle(types, flags, row_bytes):
    """Pack oracle per-position results into the product row format (include/popbam_gpu.h)."""
    L = len(types)
    counted = (flags & 2) > 0
    seg = (flags & 4) > 0
    if row_bytes == 16:
        lo, hi = (types[:, 0], types[:, 1]) if types.ndim == 2 else (types, np.zeros(L, np.uint64))
        out = np.zeros((L, 2), np.uint64)
        out[:, 0] = np.where(counted, lo, 0)
        out[:, 1] = np.where(counted, hi | (np.uint64(1) << np.uint64(62)) |
                             np.where(seg, np.uint64(1) << np.uint64(63), np.uint64(0)), 0)
        return out.view(np.uint8).reshape(-1)
    W = row_bytes * 8
    v = types.astype(np.uint64) | (np.uint64(1) << np.uint64(W - 2)) | \
        np.where(seg, np.uint64(1) << np.uint64(W - 1), np.uint64(0)).astype(np.uint64)
    v = np.where(counted, v, np.uint64(0)).astype(np.uint64)
    dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[row_bytes]
    return v.astype(dt).view(np.uint8)


def rows_to_sites(rows_u8, row_bytes, n_sites, n=64):
    """Unpack product rows -> (types, flags u8 with bit1 counted, bit2 seg); types as
    oracle_call returns them for n samples."""
    if row_bytes == 16:
        w = rows_u8.view(np.uint64).reshape(n_sites, 2)
        types, hi = w[:, 0], w[:, 1]
        counted = (hi >> np.uint64(62)) & np.uint64(1)
        seg = (hi >> np.uint64(63)) & np.uint64(1)
        if n > 64:
            types = np.stack([types, hi & np.uint64(0x3FFFFFFFFFFFFFFF)], axis=1)
    else:
        dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[row_bytes]
        v = rows_u8.view(dt).astype(np.uint64)
        W = row_bytes * 8
        counted = (v >> np.uint64(W - 2)) & np.uint64(1)
        seg = (v >> np.uint64(W - 1)) & np.uint64(1)
        types = v & ((np.uint64(1) << np.uint64(W - 2)) - np.uint64(1)) if W < 64 else v & np.uint64(0x3FFFFFFFFFFFFFFF)
    flags = (counted.astype(np.uint8) << 1) | (seg.astype(np.uint8) << 2)
    return types.astype(np.uint64), flags.astype(np.uint8)


def select_samples(batch, order):
    """A raw batch whose sample j is sample order[j] of `batch` (samples may repeat): the
    per-position read runs are regrouped in the new sample order."""
    dep = np.asarray(batch["depth"]).astype(np.int64)
    L, n = dep.shape
    start = (np.concatenate([[0], np.cumsum(dep.reshape(-1))])[:-1]).reshape(L, n)
    sel = dep[:, order]
    cnt = sel.reshape(-1)
    st = start[:, order].reshape(-1)
    seg = np.repeat(np.arange(cnt.size), cnt)
    within = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    return {"ref": np.asarray(batch["ref"]), "depth": np.ascontiguousarray(sel, dtype=np.uint16),
            "reads": np.ascontiguousarray(np.asarray(batch["reads"])[st[seg] + within], dtype=np.uint32)}


class WideSetup(Setup):
    """A golden case re-laid out for more than 64 samples (beyond the reference): its
    populations keep their order and sample order, and an extra population of copies of the
    first `n_copies` samples is inserted after population `after`, so the original populations
    straddle both 64-bit words of the masks.  Copies pass / fail and carry alleles exactly as
    their originals, so counted and segregating positions are unchanged; per-population
    statistics of the original populations equal the reference's golden values (the checks
    in test_wide_samples.py say which statistics are invariant and why)."""

    def __init__(self, case_name, args, region, n_copies=32, after=1):
        super().__init__(case_name, args, region)
        sm0 = self.sm
        order, samples, spop = [], [], []
        pops = list(sm0.pops[:after + 1]) + ["copies"] + list(sm0.pops[after + 1:])
        for p in range(len(sm0.pops)):
            for s, sp in enumerate(sm0.sample_pop):
                if sp == p:
                    order.append(s)
                    samples.append(sm0.samples[s])
                    spop.append(p if p <= after else p + 1)
            if p == after:
                for s in range(n_copies):
                    order.append(s)
                    samples.append("x" + sm0.samples[s])
                    spop.append(after + 1)
        self.order = order
        self.sm = opt.SampleModel(samples, pops, {}, spop)
        self.masks, self.pop_n = self.sm.pop_masks()
        if self.opts.flag & opt.BAM_OUTGROUP:
            self.outidx = max(i for i, s in enumerate(self.sm.samples) if s == self.opts.outgroup)
        self.batch = select_samples(self.batch, order)
        self._kbatch = None


def labelled_values(text):
    """{(line, label[name]): value} plus {(line, '#k'): k-th leading field} of a TSV."""
    out = {}
    for li, line in enumerate(text.splitlines()):
        f = line.split("\t")
        for k in range(min(4, len(f))):
            out[(li, f"#{k}")] = f[k]
        for a, b in zip(f, f[1:]):
            if a.endswith(":"):
                out[(li, a)] = b
    return out
