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
