"""ctypes binding of libpopbam_gpu.so (include/popbam_gpu.h).

The library is built in-tree by popbam_amd/csrc/Makefile (`python -c "import
__graft_entry__ as g; g.build()"`).  There is no CPU fallback: `load()` raises if the
shared object is missing, and every compute entry point fails with PBG_E_NODEV when no
HIP device is visible.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("POPBAM_GPU_LIB") or os.path.join(HERE, "libpopbam_gpu.so")

PBG_MAX_SAMPLES = 126   # 64 in the reference (u64 masks); 65..126 on two-word masks
PBG_MAX_POPS = 64
PBG_SITE_BLOCK = 64

PBG_OK, PBG_E_ARG, PBG_E_HIP, PBG_E_NOMEM, PBG_E_RANGE, PBG_E_NODEV, PBG_E_BATCH = 0, -1, -2, -3, -4, -5, -6

PBG_S_NUCDIV, PBG_S_SFS, PBG_S_ZNS, PBG_S_OMEGA, PBG_S_WALL = 0x1, 0x2, 0x4, 0x8, 0x10
PBG_S_DIV_IND, PBG_S_DIV_POP, PBG_S_HAP_K, PBG_S_HAP_EHHS, PBG_S_HAP_DXY = 0x20, 0x40, 0x80, 0x100, 0x200
PBG_S_TREE = 0x400

# every symbol include/popbam_gpu.h declares
EXPORTS = ["pbg_create", "pbg_destroy", "pbg_last_error", "pbg_row_bytes", "pbg_k_bytes", "pbg_sfs_stride",
           "pbg_device_count", "pbg_call_sites", "pbg_window_stats", "pbg_check", "pbg_run", "pbg_take_text",
           "pbg_format", "pbg_build_info", "pbg_set_kernel_timing", "pbg_kernel_time", "pbg_call_time", "pbg_synth_max_keys",
           "pbg_synth_pileup", "pbg_stream_open", "pbg_stream_push", "pbg_stream_push_compact", "pbg_stream_finish", "pbg_stream_text",
           "pbg_stream_rows", "pbg_stream_profile", "pbg_stream_error", "pbg_stream_close"]


class PbgParams(C.Structure):
    _fields_ = [("n_samples", C.c_int32), ("n_pops", C.c_int32), ("pop_mask", C.c_uint64 * PBG_MAX_POPS),
                ("pop_n", C.c_int32 * PBG_MAX_POPS), ("min_depth", C.c_int32), ("max_depth", C.c_int32),
                ("min_rmsQ", C.c_int32), ("min_snpQ", C.c_int32), ("min_mapQ", C.c_int32),
                ("min_baseQ", C.c_int32), ("flag", C.c_uint32), ("pop_mask_hi", C.c_uint64 * PBG_MAX_POPS)]

    def set_pop_mask(self, i: int, mask: int):
        """Population i's sample mask (an int of up to PBG_MAX_SAMPLES bits) -> pop_mask /
        pop_mask_hi."""
        self.pop_mask[i], self.pop_mask_hi[i] = mask & ((1 << 64) - 1), mask >> 64

    def get_pop_mask(self, i: int) -> int:
        return int(self.pop_mask[i]) | (int(self.pop_mask_hi[i]) << 64)


class PbgPileup(C.Structure):
    _fields_ = [("n_sites", C.c_uint32), ("pos0", C.c_int32), ("ref", C.c_void_p), ("k", C.c_void_p),
                ("rmsq", C.c_void_p), ("block_off", C.c_void_p), ("keys", C.c_void_p)]


class PbgSynthSpec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("contig", C.c_int32), ("mean_depth", C.c_int32), ("pos0", C.c_int64),
                ("n_sites", C.c_uint32)]


class PbgWindow(C.Structure):
    _fields_ = [("beg", C.c_int32), ("end", C.c_int32)]


class PbgStatOpts(C.Structure):
    _fields_ = [("stats", C.c_uint32), ("min_freq", C.c_int32), ("outidx", C.c_int32), ("jc", C.c_int32)]


class PbgWindowOut(C.Structure):
    _fields_ = [(nm, C.c_void_p) for nm in
                ("num_sites", "segsites", "pi", "dxy", "td", "fwh", "ld_snps", "ld_val", "ld_q", "div_ind",
                 "div_fixed", "div_seg", "div_pop", "nhaps", "hap_val", "hap_dxy", "hap_min", "tree_diff",
                 "sfs_bins", "seg_pop", "theta_w")]


class PbgCmd(C.Structure):
    _fields_ = [("cmd", C.c_int32), ("output", C.c_int32), ("min_sites", C.c_int32), ("min_snps", C.c_int32),
                ("min_freq", C.c_int32), ("outidx", C.c_int32), ("jc", C.c_int32), ("windowed", C.c_int32),
                ("win_size", C.c_int64), ("beg", C.c_int32), ("end", C.c_int32), ("chr_name", C.c_char_p),
                ("sample_names", C.POINTER(C.c_char_p)), ("pop_names", C.POINTER(C.c_char_p)),
                ("refid", C.c_char_p), ("ms_windows", C.c_int32)]


class PbgStreamProf(C.Structure):
    _fields_ = [("h2d_bytes", C.c_uint64), ("pieces", C.c_uint32), ("chunks", C.c_uint32),
                ("pinned_chunks", C.c_uint32), ("_pad", C.c_uint32), ("ms_stage", C.c_double),
                ("ms_wait", C.c_double), ("ms_h2d", C.c_double), ("ms_call", C.c_double), ("ms_finish", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "_pad"}


_lib = None


def load(torch_first: bool = True):
    """Load libpopbam_gpu.so once per process.

    One HIP runtime per process: the PyTorch ROCm wheel bundles its own libamdhip64.so.7 /
    libhsa-runtime64.so.1 and loads them under different file names.  If this library pulled
    /opt/rocm's copies in first, torch imported later would load a second HSA runtime that finds
    no GPU, so processes that use torch (tests, bench.py) import it first (torch_first) and our
    NEEDED sonames bind to its copies.  The command line never uses torch: it passes
    torch_first=False and the library runs on the system HIP runtime (no torch import, ~1-2 s of
    a fresh process), unless torch is already in the process."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           "(there is no CPU fallback)")
    if torch_first or "torch" in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    lib.pbg_create.argtypes = [P(vp), C.c_int, P(PbgParams)]
    lib.pbg_create.restype = C.c_int
    lib.pbg_destroy.argtypes = [vp]
    lib.pbg_destroy.restype = None
    lib.pbg_last_error.argtypes = [vp]
    lib.pbg_last_error.restype = C.c_char_p
    for nm in ("pbg_row_bytes", "pbg_k_bytes", "pbg_sfs_stride"):
        getattr(lib, nm).argtypes = [vp]
        getattr(lib, nm).restype = C.c_int
    lib.pbg_device_count.argtypes = []
    lib.pbg_device_count.restype = C.c_int
    lib.pbg_call_sites.argtypes = [vp, P(PbgPileup), vp, vp, vp]
    lib.pbg_call_sites.restype = C.c_int
    lib.pbg_window_stats.argtypes = [vp, vp, C.c_uint32, vp, C.c_uint32, P(PbgStatOpts), P(PbgWindowOut), vp]
    lib.pbg_window_stats.restype = C.c_int
    lib.pbg_build_info.argtypes = []
    lib.pbg_build_info.restype = C.c_char_p
    lib.pbg_check.argtypes = [vp, vp]
    lib.pbg_check.restype = C.c_int
    lib.pbg_take_text.argtypes = [vp, C.c_char_p, C.c_size_t]
    lib.pbg_take_text.restype = C.c_long
    lib.pbg_run.argtypes = [vp, P(PbgCmd), P(PbgPileup), C.c_char_p, C.c_size_t, P(C.c_size_t)]
    lib.pbg_run.restype = C.c_long
    lib.pbg_format.argtypes = [vp, P(PbgCmd), P(PbgWindowOut), C.c_uint32, vp, vp, C.c_char_p, C.c_size_t,
                               P(C.c_size_t)]
    lib.pbg_format.restype = C.c_long
    lib.pbg_set_kernel_timing.argtypes = [vp, C.c_int]
    lib.pbg_set_kernel_timing.restype = C.c_int
    lib.pbg_kernel_time.argtypes = [vp, P(C.c_double), P(C.c_uint32)]
    lib.pbg_kernel_time.restype = C.c_int
    lib.pbg_call_time.argtypes = [vp, P(C.c_double), P(C.c_uint32)]
    lib.pbg_call_time.restype = C.c_int
    lib.pbg_synth_max_keys.argtypes = [vp, P(PbgSynthSpec)]
    lib.pbg_synth_max_keys.restype = C.c_uint64
    lib.pbg_synth_pileup.argtypes = [vp, P(PbgSynthSpec), vp, vp, vp, vp, vp, C.c_uint64, P(C.c_uint64), vp]
    lib.pbg_synth_pileup.restype = C.c_int
    lib.pbg_stream_open.argtypes = [vp, P(PbgCmd), C.c_uint32, C.c_int32, C.c_uint32, C.c_uint32, P(vp)]
    lib.pbg_stream_open.restype = C.c_int
    lib.pbg_stream_push.argtypes = [vp, P(PbgPileup)]
    lib.pbg_stream_push.restype = C.c_int
    lib.pbg_stream_push_compact.argtypes = [vp, P(PbgPileup)]
    lib.pbg_stream_push_compact.restype = C.c_int
    lib.pbg_stream_finish.argtypes = [vp]
    lib.pbg_stream_finish.restype = C.c_int
    lib.pbg_stream_text.argtypes = [vp, C.c_uint32, C.c_char_p, C.c_size_t, P(C.c_size_t)]
    lib.pbg_stream_text.restype = C.c_long
    lib.pbg_stream_rows.argtypes = [vp, vp, C.c_size_t]
    lib.pbg_stream_rows.restype = C.c_int
    lib.pbg_stream_profile.argtypes = [vp, P(PbgStreamProf)]
    lib.pbg_stream_profile.restype = C.c_int
    lib.pbg_stream_error.argtypes = [vp]
    lib.pbg_stream_error.restype = C.c_char_p
    lib.pbg_stream_close.argtypes = [vp]
    lib.pbg_stream_close.restype = None
    _lib = lib
    return lib


class PbgError(RuntimeError):
    pass


class Context:
    """Owns one pbg_ctx (one device)."""

    def __init__(self, params: PbgParams, device: int = 0, torch_first: bool = True):
        self.lib = load(torch_first)
        self.h = C.c_void_p()
        rc = self.lib.pbg_create(C.byref(self.h), device, C.byref(params))
        if rc != PBG_OK:
            raise PbgError(f"pbg_create failed ({rc}): {self.lib.pbg_last_error(None).decode()}")
        self.params = params

    def check(self, rc, what):
        if rc < 0:
            raise PbgError(f"{what} failed ({rc}): {self.lib.pbg_last_error(self.h).decode()}")
        return rc

    @property
    def row_bytes(self):
        return self.lib.pbg_row_bytes(self.h)

    @property
    def k_bytes(self):
        return self.lib.pbg_k_bytes(self.h)

    @property
    def sfs_stride(self):
        return self.lib.pbg_sfs_stride(self.h)

    def sync_check(self, stream=None):
        """pbg_check: wait for `stream` and raise if a kernel flagged an inconsistent batch."""
        return self.check(self.lib.pbg_check(self.h, stream), "pbg_check")

    def close(self):
        if self.h:
            self.lib.pbg_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Stream:
    """A streamed run (pbg_stream_*): pieces of a region's HOST key batch pushed in position
    order, then every command's TSV.  `cmds` are PbgCmd structures (kept alive here)."""

    def __init__(self, ctx: Context, cmds, pos0: int, n_sites: int, chunk_sites: int = 0):
        self.ctx, self.cmds = ctx, list(cmds)
        arr = (PbgCmd * max(1, len(self.cmds)))(*self.cmds)
        self._arr = arr
        self.h = C.c_void_p()
        ctx.check(ctx.lib.pbg_stream_open(ctx.h, arr, len(self.cmds), pos0, n_sites, chunk_sites, C.byref(self.h)),
                  "pbg_stream_open")

    def push(self, piece: PbgPileup, compact: bool = False):
        """pbg_stream_push, or pbg_stream_push_compact for a compact piece (rmsq bit 31 flags the
        reference-only tasks whose keys the piece leaves out)."""
        if compact:
            self.ctx.check(self.ctx.lib.pbg_stream_push_compact(self.h, C.byref(piece)), "pbg_stream_push_compact")
        else:
            self.ctx.check(self.ctx.lib.pbg_stream_push(self.h, C.byref(piece)), "pbg_stream_push")

    def finish(self):
        self.ctx.check(self.ctx.lib.pbg_stream_finish(self.h), "pbg_stream_finish")

    def text(self, i: int) -> str:
        need = C.c_size_t(0)
        r = self.ctx.lib.pbg_stream_text(self.h, i, None, 0, C.byref(need))
        if r != PBG_E_RANGE:
            self.ctx.check(r, "pbg_stream_text")
        buf = C.create_string_buffer(max(1, need.value))
        self.ctx.check(self.ctx.lib.pbg_stream_text(self.h, i, buf, need.value, C.byref(need)), "pbg_stream_text")
        return buf.value.decode()

    def rows_into(self, ptr: int, cap: int):
        """Copy the region's rows into host or device memory at ptr (cap bytes)."""
        self.ctx.check(self.ctx.lib.pbg_stream_rows(self.h, ptr, cap), "pbg_stream_rows")

    def profile(self) -> dict:
        pr = PbgStreamProf()
        self.ctx.check(self.ctx.lib.pbg_stream_profile(self.h, C.byref(pr)), "pbg_stream_profile")
        return pr.as_dict()

    def close(self):
        if self.h:
            self.ctx.lib.pbg_stream_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
