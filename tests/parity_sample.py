"""Sampled oracle check of a full-size timed run (test infrastructure: the checker).

bench.py calls `check_windows` after its timed region: a few windows of the run are drawn at
random, their positions regenerated on the CPU (the oracle's copy of the synthetic generator,
oracle/popbam_oracle.cpp orc_synth_batch), called by the oracle's restatement of call_base ->
errmod_cal -> gl2cns -> clean_heterozygotes / segbase / qfilter (pop_utils.cpp:66-201, 280-365;
popbam.cpp:186-313), and reduced by its window loop (calc_nucdiv / calc_sfs / calc_zns /
calc_diverge / calc_ehhs ...).  The GPU's rows of those positions must equal the oracle's bit for
bit, and the GPU's window outputs, printed by the library's print_<stat> (pbg_format), must equal
the oracle's text byte for byte.  Nothing here is timed or shipped.
"""
from __future__ import annotations

import ctypes as C
import random

import numpy as np

import harness

# printed statistics per PBG_S_* flag: (popbam_func_t, -o)
CMD_OF_STAT = {0x001: (4, 0), 0x002: (6, 0), 0x004: (5, 0), 0x008: (5, 1), 0x010: (5, 2), 0x020: (2, 0),
               0x040: (2, 1), 0x080: (1, 0), 0x100: (1, 1), 0x200: (1, 2), 0x400: (3, 0)}


def _names(n, np_):
    sn = (C.c_char_p * n)(*[f"s{i}".encode() for i in range(n)])
    pn = (C.c_char_p * np_)(*[f"p{i}".encode() for i in range(np_)])
    return sn, pn


def _gpu_text(ctx, params, one: dict, cmd_id: int, output: int, L: int, min_freq: int) -> str:
    from popbam_amd import _lib
    n, np_ = params.n_samples, params.n_pops
    o = _lib.PbgWindowOut()
    keep = {}
    for k, _ in _lib.PbgWindowOut._fields_:
        if k in one:
            keep[k] = np.ascontiguousarray(one[k])
            setattr(o, k, keep[k].ctypes.data)
    c = _lib.PbgCmd()
    c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq = cmd_id, output, 10, 10, min_freq
    c.chr_name = b"chr1"
    sn, pn = _names(n, np_)
    c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
    c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
    c.refid = b"ref"
    wb, we = np.array([0], np.int32), np.array([L], np.int32)
    buf = C.create_string_buffer(1 << 20)
    need = C.c_size_t()
    ctx.check(ctx.lib.pbg_format(ctx.h, C.byref(c), C.byref(o), 1, wb.ctypes.data, we.ctypes.data, buf, 1 << 20,
                                 C.byref(need)), "pbg_format")
    return buf.value.decode()


def _oracle_text(params, types, flags, cmd_id: int, output: int, L: int, min_freq: int) -> str:
    p = harness.oracle_params_from(params)
    c = harness.OrcCmd()
    n, np_ = params.n_samples, params.n_pops
    c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq = cmd_id, output, 10, 10, min_freq
    c.chr_name = b"chr1"
    sn, pn = _names(n, np_)
    c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
    c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
    c.refid = b"ref"
    wb, we = np.array([0], np.int32), np.array([L], np.int32)
    buf = C.create_string_buffer(1 << 20)
    r = harness.oracle().orc_windows_from_sites(C.byref(p), C.byref(c), types.ctypes.data, flags.ctypes.data, 1,
                                                wb.ctypes.data, we.ctypes.data, buf, 1 << 20)
    assert r >= 0
    return buf.value.decode()


def check_windows(ctx, params, picks, seed: int, depth: int, stats: int, min_freq: int = 1) -> dict:
    """picks: [(contig, pos_lo, pos_hi, gpu_rows_u8, gpu_window_outputs)] where gpu_rows_u8 are
    the run's rows of positions [pos_lo, pos_hi) and gpu_window_outputs maps pbg_window_out
    field names to that one window's values (host arrays).  Returns a summary dict."""
    rb = ctx.row_bytes
    n = params.n_samples
    p = harness.oracle_params_from(params)
    cmds = [CMD_OF_STAT[s] for s in sorted(CMD_OF_STAT) if stats & s]
    bad = []
    positions = 0
    for contig, lo, hi, rows, one in picks:
        L = hi - lo
        positions += L
        batch = harness.synth_batch(seed, lo, hi, n, depth, params.max_depth, contig=contig)
        _, types, _, flags = harness.oracle_call(p, batch)
        want = harness.rows_from_oracle(types, flags, rb)
        if not np.array_equal(np.asarray(rows, dtype=np.uint8), want):
            diff = int(np.flatnonzero((np.asarray(rows).reshape(L, rb) != want.reshape(L, rb)).any(axis=1))[0])
            bad.append({"contig": contig, "pos": lo + diff, "what": "rows"})
            continue
        for cmd_id, output in cmds:
            g = _gpu_text(ctx, params, one, cmd_id, output, L, min_freq)
            o = _oracle_text(params, types, flags, cmd_id, output, L, min_freq)
            if g != o:
                bad.append({"contig": contig, "beg": lo, "end": hi, "cmd": cmd_id, "output": output,
                            "gpu": g[:200], "oracle": o[:200]})
    return {"ok": not bad, "windows": len(picks), "positions": positions, "commands": len(cmds),
            "mismatches": bad[:5]}


def window_slices(outs: dict, n_win: int, idx: int) -> dict:
    """The window `idx` of host pbg_window_out arrays laid out [n_win * per]."""
    one = {}
    for k, v in outs.items():
        per = v.size // max(1, n_win)
        one[k] = v[idx * per:(idx + 1) * per]
    return one


def pick(n_win: int, k: int, seed: int) -> list[int]:
    rng = random.Random(seed)
    return sorted(rng.sample(range(n_win), min(k, n_win)))
