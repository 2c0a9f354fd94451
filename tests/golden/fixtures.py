"""Golden-fixture access for the tests (test infrastructure).

Each fixture directory holds what the REFERENCE consumed (ref.fa, in.bam, in.bam.bai) and
what it printed (out/*.tsv, produced by make_golden.py with oracle/_ref/popbam).  The dense
pileup batch -- the input format of the product C-ABI -- is rebuilt here from in.bam:

  * `read_bam`   decodes BGZF/BAM (SAM spec v1) into `Read` records (file order);
  * `build_batch` restates the pileup walk of bam_pileup.c:283-407 (a position gets a
    callback iff >= 1 mask-passing read covers it, reads in file order; BAM_DEF_MASK at
    bam.h:123) and the per-sample partition of popbamData::call_base
    (popbam.cpp:220-249: skip is_del / is_refskip / unmapped, RG -> sample, keep the first
    `max_depth` reads of each sample), emitting one u32 record per kept read:
        bits 0-7 baseQ (bam1_qual[qpos]), 8-15 mapQ, 16-19 nt16 base, bit 20 strand.

The pileup's 8000-read `maxcnt` (bam_pileup.c:260, 375) is not restated: fixtures stay far
below it.
"""
from __future__ import annotations

import gzip
import json
import os
import struct
from functools import lru_cache

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CIGAR_OPS = "MIDNSHP=X"
BAM_DEF_MASK = 0x4 | 0x100 | 0x200 | 0x400


def read_bam(path):
    """Returns (header_text, [(name, len)], reads) with reads as dicts in file order."""
    with open(path, "rb") as f:
        raw = gzip.decompress(f.read())       # BGZF = concatenated gzip members
    assert raw[:4] == b"BAM\1"
    off = 4
    (l_text,) = struct.unpack_from("<i", raw, off); off += 4
    text = raw[off:off + l_text].decode(); off += l_text
    (n_ref,) = struct.unpack_from("<i", raw, off); off += 4
    refs = []
    for _ in range(n_ref):
        (ln,) = struct.unpack_from("<i", raw, off); off += 4
        name = raw[off:off + ln - 1].decode(); off += ln
        (lr,) = struct.unpack_from("<i", raw, off); off += 4
        refs.append((name, lr))
    reads = []
    end = len(raw)
    while off < end:
        (bs,) = struct.unpack_from("<i", raw, off)
        rec = raw[off + 4: off + 4 + bs]
        off += 4 + bs
        tid, pos, lname, mapq, _bin, ncig, flag, lseq = struct.unpack_from("<iiBBHHHi", rec, 0)
        p = 32 + lname
        cig = struct.unpack_from("<%dI" % ncig, rec, p); p += 4 * ncig
        seq = rec[p:p + (lseq + 1) // 2]; p += (lseq + 1) // 2
        qual = rec[p:p + lseq]; p += lseq
        aux = rec[p:]
        rg = None
        q = 0
        while q < len(aux):
            tag = aux[q:q + 2].decode(); typ = chr(aux[q + 2]); q += 3
            if typ == "Z":
                z = aux.index(b"\0", q)
                if tag == "RG":
                    rg = aux[q:z].decode()
                q = z + 1
            else:
                raise ValueError("fixture reader only supports Z tags")
        nt16 = np.empty(lseq, dtype=np.uint8)
        sb = np.frombuffer(seq, dtype=np.uint8)
        nt16[0::2] = sb[: (lseq + 1) // 2] >> 4
        nt16[1::2] = sb[: lseq // 2] & 0xF
        reads.append(dict(tid=tid, pos=pos, mapq=mapq, flag=flag,
                          cigar=[(CIGAR_OPS[c & 0xF], c >> 4) for c in cig],
                          nt16=nt16, qual=np.frombuffer(qual, dtype=np.uint8), rg=rg))
    return text, refs, reads


def parse_rg(text):
    """@RG ID/SM/PO -> (rg2sample, samples, pops, sample_pop) in first-appearance order
    (restates pop_sample.cpp:15-107 for well-formed headers)."""
    samples, pops, rg2s, spop = [], [], {}, {}
    for line in text.splitlines():
        if not line.startswith("@RG"):
            continue
        f = dict(x.split(":", 1) for x in line.split("\t")[1:] if ":" in x)
        sm, po = f["SM"], f.get("PO")
        if sm not in samples:
            samples.append(sm)
        rg2s[f["ID"]] = samples.index(sm)
        if po is not None and sm not in spop:
            if po not in pops:
                pops.append(po)
            spop[sm] = pops.index(po)
    return rg2s, samples, pops, [spop[s] for s in samples]


def build_batch(refseq: bytes, reads, rg2s, n_samples, max_depth, tid=0):
    L = len(refseq)
    covered = np.zeros(L + 1, dtype=np.int32)
    P, S, R, O = [], [], [], []
    for order, r in enumerate(reads):
        if r["tid"] != tid or (r["flag"] & BAM_DEF_MASK):
            continue
        s = rg2s[r["rg"]]
        rp, qp = r["pos"], 0
        strand = (r["flag"] >> 4) & 1
        hi = (r["mapq"] << 8) | (strand << 20)
        for op, ln in r["cigar"]:
            if op in "M=X":
                idx = np.arange(qp, qp + ln)
                P.append(np.arange(rp, rp + ln))
                R.append(r["qual"][idx].astype(np.uint32) | (r["nt16"][idx].astype(np.uint32) << 16) | hi)
                S.append(np.full(ln, s, dtype=np.int64))
                O.append(np.full(ln, order, dtype=np.int64))
                covered[rp] += 1; covered[rp + ln] -= 1
                rp += ln; qp += ln
            elif op in "DN":
                covered[rp] += 1; covered[rp + ln] -= 1
                rp += ln
            elif op in "SI":
                qp += ln
    cov = np.cumsum(covered)[:L] > 0
    ref = np.frombuffer(refseq, dtype=np.uint8).copy()
    ref[~cov] |= 0x80
    depth = np.zeros((L, n_samples), dtype=np.uint16)
    if not P:
        return dict(ref=ref, depth=depth, reads=np.zeros(0, np.uint32))
    P = np.concatenate(P); S = np.concatenate(S); R = np.concatenate(R); O = np.concatenate(O)
    key = P * n_samples + S
    idx = np.lexsort((O, key))                  # by (pos, sample), then file order
    key, R = key[idx], R[idx]
    # rank within each (pos, sample) group -> max_depth cap in pileup order
    start = np.r_[0, np.nonzero(np.diff(key))[0] + 1]
    grp = np.repeat(np.arange(len(start)), np.diff(np.r_[start, len(key)]))
    rank = np.arange(len(key)) - start[grp]
    keep = rank < max_depth
    key, R = key[keep], R[keep]
    cnt = np.bincount(key, minlength=L * n_samples)
    depth[:] = cnt.reshape(L, n_samples)
    return dict(ref=ref, depth=depth, reads=R.astype(np.uint32))


def read_fasta(path):
    seqs, name, buf = {}, None, []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith(">"):
                if name is not None:
                    seqs[name] = "".join(buf).encode()
                name, buf = line[1:].split()[0], []
            else:
                buf.append(line)
    if name is not None:
        seqs[name] = "".join(buf).encode()
    return seqs


def case_dirs():
    return sorted(d for d in os.listdir(HERE) if os.path.isfile(os.path.join(HERE, d, "meta.json")))


@lru_cache(maxsize=None)
def load_case(name):
    d = os.path.join(HERE, name)
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    text, refs, reads = read_bam(os.path.join(d, "in.bam"))
    rg2s, samples, pops, spop = parse_rg(text)
    seq = read_fasta(os.path.join(d, "ref.fa"))[refs[0][0]]
    return dict(meta=meta, dir=d, header=text, refs=refs, reads=reads, rg2s=rg2s,
                samples=samples, pops=pops, sample_pop=spop, refseq=seq)


@lru_cache(maxsize=None)
def case_batch(name, max_depth=255):
    c = load_case(name)
    return build_batch(c["refseq"], c["reads"], c["rg2s"], len(c["samples"]), max_depth)


def golden_text(name, stdout_rel):
    with open(os.path.join(HERE, name, stdout_rel)) as f:
        return f.read()
