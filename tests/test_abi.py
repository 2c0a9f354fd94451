"""The C-ABI library builds, loads and exports every symbol include/popbam_gpu.h declares.
Without a GPU, creating a context fails loudly (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

from popbam_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    txt = open(os.path.join(REPO, "include", "popbam_gpu.h")).read()
    return sorted(set(re.findall(r"\b(pbg_[a-z_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    lib = _lib.load()
    names = declared_functions()
    assert set(names) == set(_lib.EXPORTS)
    for nm in names:
        assert hasattr(lib, nm), nm


def test_create_rejects_bad_params():
    lib = _lib.load()
    p = _lib.PbgParams()
    p.n_samples, p.n_pops = _lib.PBG_MAX_SAMPLES + 1, 1
    h = C.c_void_p()
    assert lib.pbg_create(C.byref(h), 0, C.byref(p)) == _lib.PBG_E_ARG
    assert b"n_samples" in lib.pbg_last_error(None)


def test_no_device_no_fallback():
    lib = _lib.load()
    if lib.pbg_device_count() > 0:
        pytest.skip("a HIP device is visible")
    p = _lib.PbgParams()
    p.n_samples, p.n_pops = 2, 1
    p.pop_mask[0], p.pop_n[0] = 3, 2
    p.max_depth = 255
    h = C.c_void_p()
    assert lib.pbg_create(C.byref(h), 0, C.byref(p)) == _lib.PBG_E_NODEV


def test_feeder_exports_header_symbols():
    from popbam_amd import feed
    txt = open(os.path.join(REPO, "include", "popbam_feed.h")).read()
    names = sorted(set(re.findall(r"\b(pbf_[a-z_]+)\s*\(", txt)))
    assert set(names) == set(feed.EXPORTS)
    lib = feed.load()
    for nm in names:
        assert hasattr(lib, nm), nm


def test_errmod_table_file_equals_the_oracles_cal_coef():
    """popbam_amd/errmod_tables.bin (written by `make`, read by every pbg_create instead of
    recomputing ~2 M x87 expl/logl) holds exactly the oracle's cal_coef tables
    (pop_utils.cpp:203-266): fk, beta, lhet, bit for bit, after a 48-byte header."""
    import numpy as np

    import harness
    path = os.path.join(REPO, "popbam_amd", "errmod_tables.bin")
    raw = np.fromfile(path, dtype=np.uint8)
    assert raw[:8].tobytes() == b"PBGTAB01"
    n_fk, n_beta, n_lhet = np.frombuffer(raw[8:32].tobytes(), np.uint64)
    body = np.frombuffer(raw[40:].tobytes(), np.float64)
    assert (n_fk, n_beta, n_lhet) == (256, 64 * 256 * 256, 256 * 256) and body.size == n_fk + n_beta + n_lhet
    lib = harness.oracle()
    for nm, off, cnt in (("orc_fk", 0, n_fk), ("orc_beta", n_fk, n_beta), ("orc_lhet", n_fk + n_beta, n_lhet)):
        f = getattr(lib, nm)
        f.restype = C.POINTER(C.c_double)
        want = np.ctypeslib.as_array(f(), (int(cnt),))
        assert np.array_equal(body[off:off + cnt].view(np.uint64), want.view(np.uint64)), nm


def test_build_kinds():
    """The shipped library reports "product"; the PBG_BOUNDS build "bounds"; experiment switches
    (some give wrong results) cannot compile into a product build (pbg_common.h #error)."""
    assert _lib.load().pbg_build_info() == b"product"
    b = os.path.join(REPO, "popbam_amd", "variants", "bounds", "libpopbam_gpu.so")
    if os.path.exists(b):
        lib = C.CDLL(b)
        lib.pbg_build_info.restype = C.c_char_p
        assert lib.pbg_build_info() == b"bounds"
    import subprocess
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-fsyntax-only", "-x", "hip", "--offload-arch=gfx950", "-DPBG_SLOW_NONET",
                        os.path.join(REPO, "popbam_amd", "csrc", "call_kernel.hip")], capture_output=True, text=True)
    assert r.returncode != 0 and "experiment switch" in r.stderr, r.stderr[-500:]
