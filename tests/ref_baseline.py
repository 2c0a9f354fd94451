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
    """ref.fa / in.bam / in.bam.bai of positions [0, L) of contig 0 of the synthetic genome."""
    import harness
    from bamwriter import Read, write_bam, write_fasta
    os.makedirs(d, exist_ok=True)
    if os.path.exists(os.path.join(d, "in.bam.bai")):
        return d
    lib = harness.oracle()
    lib.orc_synth_genotypes.restype = None
    lib.orc_synth_genotypes.argtypes = [C.c_uint64, C.c_int32, C.c_uint64, C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p]
    ref = np.zeros(L, np.uint8)
    al = np.zeros((L, n), np.uint8)
    lib.orc_synth_genotypes(seed, 0, 0, L, n, ref.ctypes.data, al.ctypes.data)
    refseq = ref.tobytes().decode()
    bases = np.frombuffer(b"ACGT", np.uint8)
    per = n // npops
    header = ["@HD\tVN:1.0\tSO:coordinate", f"@SQ\tSN:chr1\tLN:{L}"]
    for s in range(n):
        header.append(f"@RG\tID:rg{s}\tSM:s{s}\tPO:pop{min(s // per, npops - 1)}")
    reads = []
    for s in range(n):
        for i, p in enumerate(range(s % step, L - read_len + 1, step)):
            h = (i + s) & 1
            seq = bases[(al[p:p + read_len, s] >> (2 * h)) & 3].tobytes().decode()
            reads.append(Read(name=f"r{s}_{i}", tid=0, pos=p, mapq=60, flag=16 if (i >> 1) & 1 else 0,
                              cigar=[("M", read_len)], seq=seq, qual=[40] * read_len, tags={"RG": f"rg{s}"}))
    reads.sort(key=lambda r: r.pos)
    write_fasta(os.path.join(d, "ref.fa"), [("chr1", refseq)])
    write_bam(os.path.join(d, "in.bam"), "\n".join(header) + "\n", [("chr1", L)], reads)
    return d


def _run(d: str, cmd: str, region: str, win_kb: int) -> float:
    t0 = time.perf_counter()
    subprocess.run([REF_BIN, cmd, "-f", "ref.fa", "-w", str(win_kb), "in.bam", region], cwd=d, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return time.perf_counter() - t0


def time_reference(d: str, L: int, win: int, procs: int = 1) -> dict:
    """Wall seconds of `popbam nucdiv|sfs|ld -w` over [0, L): one process per command, and
    `procs` concurrent region-sharded processes per command (whole windows per shard)."""
    win_kb = win // 1000
    one = {c: _run(d, c, "chr1", win_kb) for c in ("nucdiv", "sfs", "ld")}
    out = {"single": one, "single_total_s": sum(one.values())}
    if procs > 1:
        nw = (L - 1) // win
        per = -(-nw // procs)
        regions = [f"chr1:{a * win + 1}-{min(nw, a + per) * win + 1}" for a in range(0, nw, per)]
        par = {}
        for c in ("nucdiv", "sfs", "ld"):
            t0 = time.perf_counter()
            ps = [subprocess.Popen([REF_BIN, c, "-f", "ref.fa", "-w", str(win_kb), "in.bam", r], cwd=d,
                                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL) for r in regions]
            for p in ps:
                p.wait()
            par[c] = time.perf_counter() - t0
        out["parallel"] = par
        out["parallel_total_s"] = sum(par.values())
        out["procs"] = len(regions)
    return out
