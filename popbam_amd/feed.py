"""ctypes binding of libpopbam_feed.so (include/popbam_feed.h): the host pileup feeder.

`Bam(path).pileup(...)` returns the dense batch dict ({'ref', 'depth', 'reads', 'pos0'})
that popbam_amd.engine.run_command hands to pbg_run.  No GPU is involved here.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpopbam_feed.so")

EXPORTS = ["pbf_last_error", "pbf_open", "pbf_close", "pbf_header_text", "pbf_n_refs", "pbf_ref_name",
           "pbf_ref_len", "pbf_has_index", "pbf_pileup", "pbf_pileup_mt", "pbf_batch_free", "pbf_fasta_fetch", "pbf_free",
           "pbf_pack", "pbf_keys_free", "pbf_compact", "pbf_pileup_keys_mt", "pbf_kstream_open", "pbf_kstream_next",
           "pbf_kstream_profile", "pbf_kstream_close"]

PBF_E_RG = -4


class PbfBatch(C.Structure):
    _fields_ = [("n_sites", C.c_uint32), ("pos0", C.c_int32), ("ref", C.POINTER(C.c_uint8)),
                ("depth", C.POINTER(C.c_uint16)), ("block_off", C.POINTER(C.c_uint64)),
                ("reads", C.POINTER(C.c_uint32)), ("n_reads", C.c_uint64)]


class PbfKeys(C.Structure):
    _fields_ = [("n_sites", C.c_uint32), ("pos0", C.c_int32), ("ref", C.POINTER(C.c_uint8)), ("k", C.c_void_p),
                ("rmsq", C.POINTER(C.c_uint32)), ("block_off", C.POINTER(C.c_uint64)),
                ("keys", C.POINTER(C.c_uint16)), ("n_keys", C.c_uint64)]


class PbfProfile(C.Structure):
    _fields_ = [("t_wall", C.c_double), ("t_fetch", C.c_double), ("t_inflate", C.c_double), ("t_walk", C.c_double),
                ("t_consumer_wait", C.c_double), ("bytes_compressed", C.c_uint64), ("bytes_inflated", C.c_uint64),
                ("records", C.c_uint64), ("threads", C.c_uint32), ("pieces", C.c_uint32),
                ("crowded_pieces", C.c_uint32), ("_pad", C.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "_pad"}


class PbfFilter(C.Structure):
    _fields_ = [("min_baseQ", C.c_int32), ("min_mapQ", C.c_int32), ("illumina", C.c_int32), ("k_bytes", C.c_int32),
                ("compact", C.c_int32)]


def make_filter(min_baseQ: int, min_mapQ: int, flag: int, max_depth: int, compact: bool = False) -> PbfFilter:
    """call_base's per-read filters (popbam.cpp:266-281) and the k width for max_depth; compact:
    pieces for pbg_stream_push_compact (reference-only tasks flagged in rmsq bit 31, no keys)."""
    return PbfFilter(min_baseQ & 0xFF, min_mapQ & 0xFF, 1 if flag & 0x02 else 0, 1 if max_depth <= 255 else 2,
                     1 if compact else 0)


class FeedError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build()")
    lib = C.CDLL(LIB_PATH)
    vp, P = C.c_void_p, C.POINTER
    lib.pbf_last_error.restype = C.c_char_p
    lib.pbf_open.argtypes = [P(vp), C.c_char_p]
    lib.pbf_close.argtypes = [vp]
    lib.pbf_close.restype = None
    lib.pbf_header_text.argtypes = [vp]
    lib.pbf_header_text.restype = C.c_char_p
    lib.pbf_n_refs.argtypes = [vp]
    lib.pbf_ref_name.argtypes = [vp, C.c_int]
    lib.pbf_ref_name.restype = C.c_char_p
    lib.pbf_ref_len.argtypes = [vp, C.c_int]
    lib.pbf_ref_len.restype = C.c_int64
    lib.pbf_has_index.argtypes = [vp]
    lib.pbf_pileup.argtypes = [vp, C.c_int, C.c_int32, C.c_int32, C.c_char_p, P(C.c_char_p), P(C.c_int32),
                               C.c_int, C.c_int32, C.c_int, C.c_int, P(PbfBatch)]
    lib.pbf_pileup_mt.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                  P(C.c_char_p), P(C.c_int32), C.c_int, C.c_int32, C.c_int, C.c_int, P(PbfBatch)]
    lib.pbf_batch_free.argtypes = [P(PbfBatch)]
    lib.pbf_batch_free.restype = None
    lib.pbf_pack.argtypes = [P(PbfBatch), C.c_int, P(PbfFilter), P(PbfKeys)]
    lib.pbf_keys_free.argtypes = [P(PbfKeys)]
    lib.pbf_keys_free.restype = None
    lib.pbf_compact.argtypes = [P(PbfKeys), C.c_int, C.c_int, P(PbfKeys)]
    lib.pbf_pileup_keys_mt.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_int, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_char_p,
                                       P(C.c_char_p), P(C.c_int32), C.c_int, C.c_int32, C.c_int, C.c_int, P(PbfFilter),
                                       P(PbfKeys)]
    lib.pbf_kstream_open.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_int, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_char_p, P(C.c_char_p), P(C.c_int32), C.c_int, C.c_int32, C.c_int, C.c_int,
                                     P(PbfFilter), P(vp)]
    lib.pbf_kstream_next.argtypes = [vp, P(PbfKeys)]
    lib.pbf_kstream_profile.argtypes = [vp, P(PbfProfile)]
    lib.pbf_kstream_close.argtypes = [vp]
    lib.pbf_kstream_close.restype = None
    lib.pbf_fasta_fetch.argtypes = [C.c_char_p, C.c_char_p, P(C.c_void_p), P(C.c_int64)]
    lib.pbf_free.argtypes = [vp]
    lib.pbf_free.restype = None
    _lib = lib
    return lib


def _check(lib, rc):
    if rc < 0:
        raise FeedError(rc, lib.pbf_last_error().decode(errors="replace"))
    return rc


def fasta_fetch(path: str, name: str) -> bytes:
    lib = load()
    p = C.c_void_p()
    n = C.c_int64()
    _check(lib, lib.pbf_fasta_fetch(path.encode(), name.encode(), C.byref(p), C.byref(n)))
    try:
        return C.string_at(p, n.value)
    finally:
        lib.pbf_free(p)


def _take_keys(lib, out: PbfKeys, n_samples: int, kb: int) -> dict:
    try:
        L, pos0 = out.n_sites, out.pos0
        ref = np.ctypeslib.as_array(out.ref, (max(L, 1),))[:L].copy()
        kt = C.c_uint8 if kb == 1 else C.c_uint16
        k = np.ctypeslib.as_array(C.cast(out.k, C.POINTER(kt)), (max(L * n_samples, 1),))[:L * n_samples].copy()
        rmsq = np.ctypeslib.as_array(out.rmsq, (max(L * n_samples, 1),))[:L * n_samples].copy()
        keys = np.ctypeslib.as_array(out.keys, (max(out.n_keys, 1),))[:out.n_keys].copy()
        boff = np.ctypeslib.as_array(out.block_off, ((L + 63) // 64 + 1,)).copy()
    finally:
        lib.pbf_keys_free(C.byref(out))
    return {"ref": ref, "k": k.reshape(L, n_samples), "rmsq": rmsq.reshape(L, n_samples), "keys": keys,
            "block_off": boff, "pos0": pos0}


def pack(batch: dict, n_samples: int, flt: PbfFilter) -> dict:
    """pbf_pack: a raw batch ({'ref', 'depth', 'reads'}: the callback's per-sample partition)
    -> the key batch pbg_call_sites / pbg_run take (call_base's per-read loop applied)."""
    lib = load()
    ref = np.ascontiguousarray(batch["ref"], dtype=np.uint8)
    dep = np.ascontiguousarray(batch["depth"], dtype=np.uint16).reshape(-1)
    rd = np.ascontiguousarray(batch["reads"], dtype=np.uint32)
    if rd.size == 0:
        rd = np.zeros(1, np.uint32)
    raw = PbfBatch()
    raw.n_sites, raw.pos0 = len(ref), int(batch.get("pos0", 0))
    raw.ref = ref.ctypes.data_as(C.POINTER(C.c_uint8))
    raw.depth = dep.ctypes.data_as(C.POINTER(C.c_uint16))
    raw.block_off = None
    raw.reads = rd.ctypes.data_as(C.POINTER(C.c_uint32))
    raw.n_reads = int(np.asarray(batch["depth"], dtype=np.int64).sum())
    out = PbfKeys()
    _check(lib, lib.pbf_pack(C.byref(raw), n_samples, C.byref(flt), C.byref(out)))
    return _take_keys(lib, out, n_samples, flt.k_bytes)


def compact(keys: dict, n_samples: int, k_bytes: int) -> dict:
    """pbf_compact: a key batch ({'ref', 'k', 'rmsq', 'keys', 'block_off'}) in the compact form of
    pbg_stream_push_compact (reference-only tasks: rmsq bit 31, keys left out)."""
    lib = load()
    L = len(keys["ref"])
    ref = np.ascontiguousarray(keys["ref"], dtype=np.uint8)
    k = np.ascontiguousarray(keys["k"], dtype=np.uint8 if k_bytes == 1 else np.uint16).reshape(-1)
    rmsq = np.ascontiguousarray(keys["rmsq"], dtype=np.uint32).reshape(-1)
    ks = np.ascontiguousarray(keys["keys"], dtype=np.uint16)
    if ks.size == 0:
        ks = np.zeros(1, np.uint16)
    boff = np.ascontiguousarray(keys["block_off"], dtype=np.uint64)
    src = PbfKeys()
    src.n_sites, src.pos0 = L, int(keys.get("pos0", 0))
    src.ref = ref.ctypes.data_as(C.POINTER(C.c_uint8))
    src.k = k.ctypes.data
    src.rmsq = rmsq.ctypes.data_as(C.POINTER(C.c_uint32))
    src.block_off = boff.ctypes.data_as(C.POINTER(C.c_uint64))
    src.keys = ks.ctypes.data_as(C.POINTER(C.c_uint16))
    src.n_keys = int(boff[(L + 63) // 64] - boff[0])
    out = PbfKeys()
    _check(lib, lib.pbf_compact(C.byref(src), n_samples, k_bytes, C.byref(out)))
    return _take_keys(lib, out, n_samples, k_bytes)


class Bam:
    def __init__(self, path: str):
        self.lib = load()
        self.h = C.c_void_p()
        _check(self.lib, self.lib.pbf_open(C.byref(self.h), path.encode()))
        self.path = path

    @property
    def header_text(self) -> str:
        return self.lib.pbf_header_text(self.h).decode(errors="replace")

    @property
    def refs(self):
        return [(self.lib.pbf_ref_name(self.h, i).decode(), self.lib.pbf_ref_len(self.h, i))
                for i in range(self.lib.pbf_n_refs(self.h))]

    @property
    def has_index(self) -> bool:
        return bool(self.lib.pbf_has_index(self.h))

    def pileup(self, tid: int, beg: int, end: int, refseq: bytes, rg2s: dict, n_samples: int, max_depth: int,
               fallback_sample: int = -1, threads: int = 1, chunk: int = 1 << 20, win: int = 0) -> dict:
        """Dense pileup batch of [beg, end).  threads = 1: one walk of the region (pbf_pileup).
        threads > 1: pbf_pileup_mt (chunk-position pieces walked in parallel, each thread with
        its own file handle), the pileup of the reference's walks of windows of `win`
        positions from beg (win = 0: one walk of the region, the same batch as threads = 1)."""
        ids = list(rg2s)
        rg = (C.c_char_p * max(1, len(ids)))(*[i.encode() for i in ids])
        sm = (C.c_int32 * max(1, len(ids)))(*[rg2s[i] for i in ids])
        if len(refseq) < end:
            raise FeedError(-3, "reference sequence shorter than the region")
        out = PbfBatch()
        if threads > 1:
            _check(self.lib, self.lib.pbf_pileup_mt(self.path.encode(), threads, chunk, tid, beg, end, win, refseq, rg, sm,
                                                    len(ids), fallback_sample, n_samples, max_depth, C.byref(out)))
        else:
            _check(self.lib, self.lib.pbf_pileup(self.h, tid, beg, end, refseq, rg, sm, len(ids), fallback_sample,
                                                 n_samples, max_depth, C.byref(out)))
        try:
            L = out.n_sites
            ref = np.ctypeslib.as_array(out.ref, (max(L, 1),))[:L].copy()
            depth = np.ctypeslib.as_array(out.depth, (max(L * n_samples, 1),))[:L * n_samples].copy()
            reads = np.ctypeslib.as_array(out.reads, (max(out.n_reads, 1),))[:out.n_reads].copy()
            boff = np.ctypeslib.as_array(out.block_off, ((L + 63) // 64 + 1,)).copy()
        finally:
            self.lib.pbf_batch_free(C.byref(out))
        return {"ref": ref, "depth": depth.reshape(L, n_samples), "reads": reads, "block_off": boff, "pos0": beg}

    def pileup_keys(self, tid: int, beg: int, end: int, refseq: bytes, rg2s: dict, n_samples: int, max_depth: int,
                    flt: PbfFilter, fallback_sample: int = -1, threads: int = 1, chunk: int = 1 << 20,
                    win: int = 0) -> dict:
        """Key batch of [beg, end) (pbf_pileup_keys_mt): pileup + partition + call_base's
        per-read loop, pieces walked and packed by `threads` threads; `win` as in pileup()."""
        ids = list(rg2s)
        rg = (C.c_char_p * max(1, len(ids)))(*[i.encode() for i in ids])
        sm = (C.c_int32 * max(1, len(ids)))(*[rg2s[i] for i in ids])
        if len(refseq) < end:
            raise FeedError(-3, "reference sequence shorter than the region")
        out = PbfKeys()
        _check(self.lib, self.lib.pbf_pileup_keys_mt(self.path.encode(), max(1, threads), chunk, tid, beg, end, win, refseq,
                                                     rg, sm, len(ids), fallback_sample, n_samples, max_depth,
                                                     C.byref(flt), C.byref(out)))
        return _take_keys(self.lib, out, n_samples, flt.k_bytes)

    def key_stream(self, tid: int, beg: int, end: int, refseq: bytes, rg2s: dict, n_samples: int, max_depth: int,
                   flt: PbfFilter, fallback_sample: int = -1, threads: int = 1, chunk: int = 1 << 20,
                   win: int = 0) -> "KeyStream":
        """pbf_kstream_*: the key batch of [beg, end) as pieces in position order, walked ahead by
        `threads` workers."""
        return KeyStream(self, tid, beg, end, refseq, rg2s, n_samples, max_depth, flt, fallback_sample, threads,
                         chunk, win)

    def close(self):
        if self.h:
            self.lib.pbf_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KeyStream:
    """Iterates the pieces (PbfKeys, library-owned: `release` each) of a region's key batch."""

    def __init__(self, bam: Bam, tid, beg, end, refseq, rg2s, n_samples, max_depth, flt, fallback_sample, threads,
                 chunk, win):
        self.lib = bam.lib
        if len(refseq) < end:
            raise FeedError(-3, "reference sequence shorter than the region")
        ids = list(rg2s)
        self._keep = (refseq, (C.c_char_p * max(1, len(ids)))(*[i.encode() for i in ids]),
                      (C.c_int32 * max(1, len(ids)))(*[rg2s[i] for i in ids]), flt)
        self.h = C.c_void_p()
        _check(self.lib, self.lib.pbf_kstream_open(bam.path.encode(), max(1, threads), chunk, tid, beg, end, win, refseq,
                                                   self._keep[1], self._keep[2], len(ids), fallback_sample, n_samples,
                                                   max_depth, C.byref(flt), C.byref(self.h)))

    def next(self) -> PbfKeys | None:
        p = PbfKeys()
        r = _check(self.lib, self.lib.pbf_kstream_next(self.h, C.byref(p)))
        return p if r == 1 else None

    def release(self, p: PbfKeys):
        self.lib.pbf_keys_free(C.byref(p))

    def profile(self) -> dict:
        pr = PbfProfile()
        _check(self.lib, self.lib.pbf_kstream_profile(self.h, C.byref(pr)))
        return pr.as_dict()

    def close(self):
        if self.h:
            self.lib.pbf_kstream_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
