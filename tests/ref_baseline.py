"""CPU baseline with POPBAM itself (test infrastructure, used by bench.py's
cpu_baseline leg only).

The reference binary (oracle/_ref/popbam, built from /root/reference by oracle/Makefile) runs
on a BAM written from the same counter-based synthetic genome the GPU benchmark uses: the
genotypes behind the pileup (oracle orc_synth_genotypes: reference base and two haplotype
alleles per (position, sample)), 100 bp reads every 10 bp per sample (depth 10), baseQ 40,
mapQ 60, 2 contiguous populations -- every call unambiguous.  nucdiv, sfs and
ld run as three separate processes (the reference computes each statistic in its own pass,
re-reading and re-calling every position) and their wall times are summed.  The all-core
figure runs P region-sharded processes per command concurrently (shards of whole windows).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
REF_BIN = os.path.join(REPO, "oracle", "_ref", "popbam")


def available() -> bool:
    return os.path.exists(REF_BIN) and os.access(REF_BIN, os.X_OK)


def make_inputs(d: str, seed: int, L: int, n: int, npops: int = 2, read_len: int = 100, step: int = 10) -> str:
    """ref.fa / in.bam / in.bam.bai of positions [0, L) of contig 0 of the synthetic genome
    (oracle/synth_bam.cpp: the genotypes behind the benchmark's pileup, 100 bp reads every 10 bp
    per sample, baseQ 40, mapQ 60, BGZF members compressed on several threads)."""
    import harness
    os.makedirs(d, exist_ok=True)
    if os.path.exists(os.path.join(d, "in.bam.bai")):
        return d
    lib = harness.oracle()
    lib.orc_write_synth_bam.restype = C.c_int
    lib.orc_write_synth_bam.argtypes = [C.c_char_p, C.c_uint64, C.c_uint32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                        C.c_int32]
    threads = max(1, min(16, os.cpu_count() or 1))
    rc = lib.orc_write_synth_bam(d.encode(), seed, L, n, npops, read_len, step, threads)
    if rc != 0:
        raise RuntimeError(f"orc_write_synth_bam failed ({rc})")
    return d


def _run(d: str, cmd: str, region: str, win_kb: int) -> float:
    t0 = time.perf_counter()
    subprocess.run([REF_BIN, cmd, "-f", "ref.fa", "-w", str(win_kb), "in.bam", region], cwd=d, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return time.perf_counter() - t0


def time_reference(d: str, L: int, win: int, procs: int = 1, single: bool = True, capture: bool = False) -> dict:
    """Wall seconds of `popbam nucdiv|sfs|ld -w` over [0, L): one process per command (single),
    and `procs` concurrent region-sharded processes per command (whole windows per shard; with
    capture, their stdout concatenated in shard order = the command's text)."""
    win_kb = win // 1000
    out = {}
    if single:
        one = {c: _run(d, c, "chr1", win_kb) for c in ("nucdiv", "sfs", "ld")}
        out.update({"single": one, "single_total_s": sum(one.values())})
    if procs > 1:
        nw = (L - 1) // win
        per = -(-nw // procs)
        regions = [f"chr1:{a * win + 1}-{min(nw, a + per) * win + 1}" for a in range(0, nw, per)]
        par, texts = {}, {}
        for c in ("nucdiv", "sfs", "ld"):
            t0 = time.perf_counter()
            ps = [subprocess.Popen([REF_BIN, c, "-f", "ref.fa", "-w", str(win_kb), "in.bam", r], cwd=d,
                                   stdout=subprocess.PIPE if capture else subprocess.DEVNULL,
                                   stderr=subprocess.DEVNULL) for r in regions]
            outs = [p.communicate()[0] if capture else p.wait() for p in ps]
            par[c] = time.perf_counter() - t0
            if capture:
                texts[c] = b"".join(outs).decode()
        out["parallel"] = par
        out["parallel_total_s"] = sum(par.values())
        out["procs"] = len(regions)
        if capture:
            out["texts"] = texts
    return out
