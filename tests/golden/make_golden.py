#!/usr/bin/env python3
"""Generate the golden fixtures (test infrastructure; run in the build container only).

For every scenario below this script
  1. simulates diploid samples + reads and writes ref.fa / in.bam / in.bam.bai with
     tests/golden/bamwriter.py;
  2. runs the REFERENCE popbam (oracle/_ref/popbam, built from /root/reference sources by
     oracle/Makefile) on them and stores its stdout verbatim as <case>/out/<n>.tsv;
  3. restates the pileup stage (bam_pileup.c:283-407 position walk + popbam.cpp:220-249
     per-sample partition with the max_depth cap) in Python and stores the resulting
     dense pileup batch and checks it equals what tests/golden/fixtures.py rebuilds from
     in.bam at test time (the exact input format of the product C-ABI,
     include/popbam_gpu.h `pbg_pileup`).

The reference is never needed at test time: tests read the committed fixtures.

Usage:  python tests/golden/make_golden.py [case ...]
        python tests/golden/make_golden.py --append [case ...]   (new commands only)
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from bamwriter import Read, write_bam, write_fasta  # noqa: E402

REF_BIN = os.path.join(REPO, "oracle", "_ref", "popbam")
BASES = "ACGT"
NT16 = {"A": 1, "C": 2, "G": 4, "T": 8, "N": 15}
BAM_DEF_MASK = 0x4 | 0x100 | 0x200 | 0x400   # bam.h:123 (UNMAP|SECONDARY|QCFAIL|DUP)

# ----------------------------------------------------------------------------------------
# scenarios
# ----------------------------------------------------------------------------------------
def _samples(n, pops):
    """n samples, pops = list of population names cycled contiguously."""
    per = n // len(pops)
    out = []
    for i in range(n):
        out.append((f"s{i}", pops[min(i // per, len(pops) - 1)]))
    return out


def _std_cmds(w, extra=()):
    cmds = [
        ["nucdiv", "-w", w], ["sfs", "-w", w], ["ld", "-w", w], ["ld", "-w", w, "-o", "1"],
        ["ld", "-w", w, "-o", "2"], ["ld", "-w", w, "-e"],
        ["diverge", "-w", w], ["diverge", "-w", w, "-d", "jc"], ["diverge", "-w", w, "-o", "1"],
        ["diverge", "-w", w, "-o", "1", "-t"],
        ["haplo", "-w", w], ["haplo", "-w", w, "-o", "1"], ["haplo", "-w", w, "-o", "2"],
        ["snp"],
    ]
    return cmds + [list(c) for c in extra]


SCENARIOS = {
    # G1: 12 samples, 2 contiguous populations, depth 10
    "g01_base": dict(seed=101, L=30000, samples=_samples(12, ["popA", "popB"]), step=10,
                     mu=0.02, cmds=_std_cmds("1", [["nucdiv", "-w", "10"], ["sfs", "-w", "10"],
                                                   ["ld", "-w", "10"], ["nucdiv"], ["sfs"], ["ld"],
                                                   ["nucdiv", "-w", "2", "-k", "500"],
                                                   ["tree", "-w", "1"], ["tree", "-w", "1", "-d", "jc"], ["tree"],
                                                   ["tree", "-w", "10"], ["tree", "-w", "2", "-k", "500"]])),
    # G2: interleaved population labels (Dxy asymmetry quirk)
    "g02_interleaved": dict(seed=202, L=12000, samples=[(f"s{i}", ["popA", "popB"][i % 2]) for i in range(12)],
                            step=10, mu=0.02, cmds=_std_cmds("1")),
    # G3: three populations
    "g03_threepops": dict(seed=303, L=12000, samples=_samples(12, ["p1", "p2", "p3"]), step=10,
                          mu=0.03, cmds=_std_cmds("1") + [["tree", "-w", "1"]]),
    # G4: sfs / diverge / snp with an outgroup flip
    "g04_outgroup": dict(seed=404, L=12000, samples=_samples(12, ["popA", "popB"]), step=10, mu=0.03,
                         cmds=[["sfs", "-w", "1", "-p", "s11"], ["sfs", "-w", "1", "-p", "s0"],
                               ["diverge", "-w", "1", "-o", "1", "-p", "s3"], ["sfs", "-w", "1"]]),
    # G5: low depth, low quality -> hom-alt reverts (segbase borrow quirk) and het cleaning
    "g05_lowdepth": dict(seed=505, L=12000, samples=_samples(12, ["popA", "popB"]), step=30, mu=0.05,
                         baseq=[12, 15, 18, 20, 22, 25, 30], err=0.03,
                         cmds=_std_cmds("1", [["nucdiv", "-w", "1", "-s", "9"], ["snp", "-s", "9"],
                                              ["snp", "-m", "2"], ["nucdiv", "-w", "1", "-m", "2"],
                                              ["tree", "-w", "1"], ["tree", "-w", "1", "-m", "2", "-s", "9"]])),
    # G6: lowercase soft-masked reference stretch + an N stretch
    "g06_softmask": dict(seed=606, L=12000, samples=_samples(12, ["popA", "popB"]), step=10, mu=0.02,
                         lower=[(3000, 6500)], nrun=[(9000, 9400)], cmds=_std_cmds("1")),
    # G7: multi-allelic sites (fq = -1: counted, not segregating)
    "g07_multiallelic": dict(seed=707, L=12000, samples=_samples(12, ["popA", "popB"]), step=10, mu=0.04,
                             multi=0.3, cmds=_std_cmds("1")),
    # G8: base/map quality filters, deletions, ref-skips, clips, insertions, flagged reads, mapQ spread
    "g08_filters": dict(seed=808, L=12000, samples=_samples(12, ["popA", "popB"]), step=8, mu=0.02,
                        baseq=[5, 10, 13, 20, 30, 40], mapq=[0, 10, 13, 20, 29, 37, 45, 60, 60, 60],
                        indel=0.15, flagged=0.05,
                        cmds=_std_cmds("1", [["nucdiv", "-w", "1", "-a", "7"], ["nucdiv", "-w", "1", "-b", "5"],
                                             ["sfs", "-w", "1", "-q", "40"], ["nucdiv", "-w", "1", "-i"],
                                             ["nucdiv", "-w", "1", "-a", "20"]])),
    # G9: whole-contig (no window) with > 65535 pairwise differences (u16 wrap)
    "g09_u16wrap": dict(seed=909, L=300000, samples=_samples(4, ["popA", "popB"]), step=25, mu=0.6,
                        freq_hi=True, baseq=[40], cmds=[["nucdiv", "-m", "2"], ["haplo", "-o", "2", "-m", "2"],
                                                        ["diverge", "-m", "2"], ["diverge", "-o", "1", "-m", "2"],
                                                        ["nucdiv"], ["tree", "-m", "2"], ["tree", "-m", "2", "-d", "jc"]]),
    # G10: deep pileup with -x > 255 (ks_shuffle rotation + truncation to 255 keys)
    "g10_deep": dict(seed=1010, L=2500, samples=_samples(4, ["popA", "popB"]), step=0.2, mu=0.05,
                     read_len=60, cmds=[["nucdiv", "-x", "900"], ["snp", "-x", "900"], ["snp"],
                                        ["nucdiv", "-x", "300", "-m", "280"]]),
    # G11: 11 samples (stand-in for the trial.bam config), 10 kb windows
    "g11_eleven": dict(seed=1111, L=40000, samples=_samples(11, ["mel", "sim"]), step=10, mu=0.015,
                       cmds=_std_cmds("10") + [["tree", "-w", "10"], ["tree", "-w", "5", "-d", "jc"]]),
    # G12: region forms chr:a-b, chr:a, and windows not aligned to the contig start
    "g12_regions": dict(seed=1212, L=15000, samples=_samples(8, ["popA", "popB"]), step=10, mu=0.03,
                        cmds=[["nucdiv", "REGION=chr1:2001-9000"], ["nucdiv", "-w", "1", "REGION=chr1:1,501-12,000"],
                              ["sfs", "-w", "2", "REGION=chr1:777-14777"], ["ld", "-w", "1", "REGION=chr1:5001-11000"],
                              ["nucdiv", "REGION=chr1:5000"], ["nucdiv", "-w", "3", "REGION=chr1:3001-12000"],
                              ["snp", "REGION=chr1:4001-4800"], ["nucdiv", "-w", "1", "-m", "0", "-q", "0"],
                              ["sfs", "-w", "1", "-m", "0", "-q", "0"], ["snp", "-m", "0", "-q", "0", "REGION=chr1:6500-8500"],
                              # -x 0 keeps no read (qfilter fails unless -m 0 -q 0); -x beyond 65535
                              ["nucdiv", "-w", "1", "-x", "0"], ["nucdiv", "-w", "1", "-x", "0", "-m", "0", "-q", "0"],
                              ["sfs", "-w", "2", "-x", "70000"]],
                        gap=[(7000, 7600)]),
    # G13: snp output formats -o 1 (SweepFinder) / -o 2 (ms), windows, outgroup flip, 3 populations
    "g13_snpformats": dict(seed=1313, L=12000, samples=_samples(12, ["p1", "p2", "p3"]), step=10, mu=0.03,
                           cmds=[["snp", "-o", "1"], ["snp", "-o", "2"], ["snp", "-o", "1", "-w", "2"],
                                 ["snp", "-o", "2", "-w", "2"], ["snp", "-o", "1", "-p", "s3"],
                                 ["snp", "-o", "2", "-w", "3", "-p", "s3"], ["snp", "-o", "2", "REGION=chr1:2001-5000"],
                                 ["snp", "-o", "1", "-w", "1", "REGION=chr1:2501-9000"]]),
    # G14: one population (ms header without -I)
    "g14_onepop": dict(seed=1414, L=6000, samples=_samples(6, ["solo"]), step=10, mu=0.03,
                       cmds=[["snp", "-o", "2"], ["snp", "-o", "2", "-w", "1"], ["snp", "-o", "1"], ["nucdiv", "-w", "1"],
                             ["tree", "-w", "1"], ["tree", "REGION=chr1:1001-4000"]]),
    # G15: 24 samples in 3 populations (configs[3]'s sample count: 4-byte rows, r^2 tables of
    # 3 x 9^3 entries; 1 kb and 10 kb windows)
    "g15_24s3p": dict(seed=1515, L=25000, samples=_samples(24, ["pa", "pb", "pc"]), step=10, mu=0.03,
                      cmds=_std_cmds("1", [["nucdiv", "-w", "10"], ["sfs", "-w", "10"], ["ld", "-w", "10"],
                                           ["ld", "-w", "10", "-o", "1"], ["ld", "-w", "10", "-o", "2"],
                                           ["diverge", "-w", "10"], ["diverge", "-w", "10", "-o", "1"],
                                           ["haplo", "-w", "10", "-o", "1"], ["sfs", "-w", "1", "-p", "s23"],
                                           ["tree", "-w", "5"], ["snp", "-o", "1", "-w", "1"], ["snp", "-o", "2", "-w", "2"]])),
    # G16: 24 samples in 2 populations (r^2 tables 2 x 13^3 = 4394 doubles: beyond the LDS copy)
    "g16_24s2p": dict(seed=1616, L=20000, samples=_samples(24, ["popA", "popB"]), step=10, mu=0.03,
                      cmds=_std_cmds("1", [["nucdiv", "-w", "10"], ["sfs", "-w", "10"], ["ld", "-w", "10"],
                                           ["ld", "-w", "10", "-e"], ["ld", "-w", "10", "-o", "1"]])),
    # G17: 48 samples in 2 populations (8-byte rows)
    "g17_48s": dict(seed=1717, L=10000, samples=_samples(48, ["popA", "popB"]), step=10, mu=0.03,
                    cmds=_std_cmds("1", [["nucdiv", "-w", "5"], ["ld", "-w", "5"], ["tree", "-w", "2"]])),
    # G18: 64 samples in 4 populations (16-byte rows; the reference's sample limit)
    "g18_64s4p": dict(seed=1818, L=8000, samples=_samples(64, ["q1", "q2", "q3", "q4"]), step=10, mu=0.03,
                      cmds=_std_cmds("1", [["nucdiv", "-w", "4"], ["sfs", "-w", "4"], ["ld", "-w", "4"],
                                           ["haplo", "-w", "2", "-o", "2"]])),
}


# ----------------------------------------------------------------------------------------
# simulation
# ----------------------------------------------------------------------------------------
def simulate(sc):
    rng = np.random.RandomState(sc["seed"])
    L = sc["L"]
    samples = sc["samples"]
    n = len(samples)
    read_len = sc.get("read_len", 100)
    refseq = np.array(list(rng.choice(list(BASES), size=L)))
    # genotypes: per site per sample two alleles (0..3 base indices)
    ref_idx = np.array([BASES.index(c) for c in refseq])
    geno = np.repeat(ref_idx[:, None, None], n, axis=1).repeat(2, axis=2)  # L x n x 2
    snp = rng.rand(L) < sc.get("mu", 0.02)
    for p in np.nonzero(snp)[0]:
        d = (ref_idx[p] + rng.randint(1, 4)) % 4
        f = rng.uniform(0.5, 1.0) if sc.get("freq_hi") else rng.uniform(0.0, 1.0)
        alle = rng.rand(n, 2) < f
        geno[p][alle] = d
        if rng.rand() < sc.get("multi", 0.0):
            d2 = (d + rng.randint(1, 3)) % 4
            if d2 == ref_idx[p]:
                d2 = (d2 + 1) % 4
            who = rng.rand(n, 2) < 0.3
            geno[p][who] = d2
    # soft-masking / N runs (affects the reference only)
    for a, b in sc.get("lower", []):
        for i in range(a, b):
            refseq[i] = refseq[i].lower()
    for a, b in sc.get("nrun", []):
        refseq[a:b] = "N"
    baseq = sc.get("baseq", [25, 30, 35, 40])
    mapq = sc.get("mapq", [60])
    err = sc.get("err", 0.01)
    indel = sc.get("indel", 0.0)
    flagged = sc.get("flagged", 0.0)
    step = sc["step"]
    reads = []
    rg_of = {}
    for si, (sname, _) in enumerate(samples):
        rg_of[si] = [f"rg{si}"] + ([f"rg{si}b"] if si % 3 == 0 else [])
        x = float(rng.randint(0, max(1, int(step))))
        k = 0
        while x < L - 5:
            pos = int(x)
            x += step * rng.uniform(0.5, 1.5) if step >= 1 else step
            rl = min(read_len, L - pos)
            if rl < 10:
                break
            if any(pos < gb and pos + rl > ga for ga, gb in sc.get("gap", [])):
                continue
            cigar = [("M", rl)]
            r = rng.rand() if rl >= 40 else 1.0
            if r < indel * 0.25:
                a = rng.randint(10, rl - 10)
                cigar = [("M", a), ("D", int(rng.randint(1, 4))), ("M", rl - a)]
            elif r < indel * 0.5:
                a = rng.randint(10, rl - 10)
                cigar = [("M", a), ("N", int(rng.randint(20, 200))), ("M", rl - a)]
            elif r < indel * 0.75:
                a = int(rng.randint(1, 6))
                cigar = [("S", a), ("M", rl - a)]
            elif r < indel:
                a = rng.randint(10, rl - 10)
                ins = int(rng.randint(1, 4))
                cigar = [("M", a), ("I", ins), ("M", rl - a - ins)]
            # build the read sequence along the cigar
            h = rng.randint(0, 2)
            seq, qual = [], []
            rp = pos
            for op, ln in cigar:
                if op == "M":
                    for j in range(ln):
                        if rp >= L:
                            break
                        b = geno[rp, si, h]
                        if rng.rand() < err:
                            b = (b + rng.randint(1, 4)) % 4
                        c = BASES[b] if rng.rand() > 0.002 else "N"
                        seq.append(c)
                        qual.append(int(rng.choice(baseq)))
                        rp += 1
                elif op in "DN":
                    rp += ln
                elif op in "SI":
                    for j in range(ln):
                        seq.append(BASES[rng.randint(0, 4)])
                        qual.append(int(rng.choice(baseq)))
            # trim cigar if the read ran off the contig end
            span = sum(l for o, l in cigar if o in "MDN")
            if pos + span > L:
                continue
            flag = 16 if rng.rand() < 0.5 else 0
            if rng.rand() < flagged:
                flag |= int(rng.choice([0x100, 0x200, 0x400, 0x4]))
            rg = rg_of[si][k % len(rg_of[si])]
            k += 1
            reads.append(Read(name=f"r{si}_{k}", tid=0, pos=pos, mapq=int(rng.choice(mapq)), flag=flag,
                              cigar=cigar, seq="".join(seq), qual=qual, tags={"RG": rg}))
    # stable sort by position keeps per-sample emission order for equal positions;
    # interleave samples deterministically
    reads.sort(key=lambda r: (r.tid, r.pos))
    return "".join(refseq), reads, rg_of


def header_text(L, samples, rg_of):
    lines = ["@HD\tVN:1.0\tSO:coordinate", f"@SQ\tSN:chr1\tLN:{L}\tAS:simref"]
    for si, (sname, pop) in enumerate(samples):
        for rg in rg_of[si]:
            lines.append(f"@RG\tID:{rg}\tSM:{sname}\tPO:{pop}")
    return "\n".join(lines) + "\n"


# ----------------------------------------------------------------------------------------
# pileup restatement -> dense batch (the C-ABI input format)
# ----------------------------------------------------------------------------------------
def build_batch(refseq, reads, samples, rg_of, max_depth):
    """Restates bam_pileup.c (positions with >=1 mask-passing read get a callback; reads in
    file order) and popbamData::call_base's partition (popbam.cpp:220-249: skip is_del /
    is_refskip / FUNMAP, RG -> sample, keep the first max_depth reads per sample)."""
    L = len(refseq)
    n = len(samples)
    rg2s = {rg: si for si, rgs in rg_of.items() for rg in rgs}
    covered = np.zeros(L, dtype=bool)
    per_pos = [[] for _ in range(L)]        # list of (sample, record) in pileup order
    for r in reads:
        if r.tid < 0 or (r.flag & BAM_DEF_MASK):
            continue
        rp, qp = r.pos, 0
        for op, ln in r.cigar:
            if op in "M=X":
                for j in range(ln):
                    covered[rp] = True
                    c = r.seq[qp]
                    rec = (r.qual[qp] & 0xFF) | (r.mapq << 8) | (NT16.get(c, 15) << 16) | (((r.flag >> 4) & 1) << 20)
                    per_pos[rp].append((rg2s[r.tags["RG"]], rec))
                    rp += 1
                    qp += 1
            elif op in "DN":
                covered[rp:rp + ln] = True      # in the pileup as is_del / is_refskip, skipped by call_base
                rp += ln
            elif op in "SI":
                qp += ln
    depth = np.zeros((L, n), dtype=np.uint16)
    recs = []
    for p in range(L):
        buckets = [[] for _ in range(n)]
        for s, rec in per_pos[p]:
            if len(buckets[s]) < max_depth:
                buckets[s].append(rec)
        for s in range(n):
            depth[p, s] = len(buckets[s])
            recs.extend(buckets[s])
    ref = np.frombuffer(refseq.encode(), dtype=np.uint8).copy()
    ref[~covered] |= 0x80          # no pileup callback at this position
    return dict(ref=ref, depth=depth, reads=np.array(recs, dtype=np.uint32))


# ----------------------------------------------------------------------------------------
def run_case(name, sc):
    d = os.path.join(HERE, name)
    if os.path.isdir(d):
        shutil.rmtree(d)
    os.makedirs(os.path.join(d, "out"))
    refseq, reads, rg_of = simulate(sc)
    samples = sc["samples"]
    write_fasta(os.path.join(d, "ref.fa"), [("chr1", refseq)])
    write_bam(os.path.join(d, "in.bam"), header_text(sc["L"], samples, rg_of), [("chr1", sc["L"])], reads)
    meta = dict(samples=[s for s, _ in samples], pops=[p for _, p in samples], L=sc["L"], cases=[])
    xs = set()
    for i, cmd in enumerate(sc["cmds"]):
        region = "chr1"
        args = []
        for a in cmd:
            if a.startswith("REGION="):
                region = a[len("REGION="):]
            else:
                args.append(a)
        full = [REF_BIN, args[0], "-f", "ref.fa"] + args[1:] + ["in.bam", region]
        res = subprocess.run(full, cwd=d, capture_output=True, text=True, timeout=600)
        out = f"out/{i:02d}_{args[0]}.tsv"
        with open(os.path.join(d, out), "w") as f:
            f.write(res.stdout)
        x = 255
        if "-x" in args:
            x = int(args[args.index("-x") + 1])
        xs.add(x)
        meta["cases"].append(dict(args=args, region=region, stdout=out, rc=res.returncode,
                                  max_depth=x, stderr=res.stderr[-400:]))
        print(f"  {name} {' '.join(args)} {region}: rc={res.returncode} lines={res.stdout.count(chr(10))}")
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    fai = os.path.join(d, "ref.fa.fai")
    if os.path.exists(fai):
        os.remove(fai)
    # cross-check: the test-time batch builder (fixtures.py, decodes in.bam) must agree
    # with this script's own restatement on the simulated read list.
    import fixtures
    fixtures.load_case.cache_clear(); fixtures.case_batch.cache_clear()
    for x in sorted(xs):
        b = build_batch(refseq, reads, samples, rg_of, x)
        c = fixtures.case_batch(name, x)
        for k in ("ref", "depth", "reads"):
            assert np.array_equal(b[k], c[k]), (name, x, k)


def append_cases(name, sc):
    """Run only the commands added to a scenario after its fixtures were made (same BAM,
    existing outputs untouched; new outputs get the next indices)."""
    d = os.path.join(HERE, name)
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    for i, cmd in enumerate(sc["cmds"]):
        if i < len(meta["cases"]):
            continue
        region = "chr1"
        args = []
        for a in cmd:
            if a.startswith("REGION="):
                region = a[len("REGION="):]
            else:
                args.append(a)
        full = [REF_BIN, args[0], "-f", "ref.fa"] + args[1:] + ["in.bam", region]
        res = subprocess.run(full, cwd=d, capture_output=True, text=True, timeout=600)
        out = f"out/{i:02d}_{args[0]}.tsv"
        with open(os.path.join(d, out), "w") as f:
            f.write(res.stdout)
        x = int(args[args.index("-x") + 1]) if "-x" in args else 255
        meta["cases"].append(dict(args=args, region=region, stdout=out, rc=res.returncode,
                                  max_depth=x, stderr=res.stderr[-400:]))
        print(f"  {name} {' '.join(args)} {region}: rc={res.returncode} lines={res.stdout.count(chr(10))}")
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    fai = os.path.join(d, "ref.fa.fai")
    if os.path.exists(fai):
        os.remove(fai)


def main(argv):
    if not os.path.exists(REF_BIN):
        sys.exit("build the reference first: make -C oracle ref")
    if argv and argv[0] == "--append":
        for nm in argv[1:] or list(SCENARIOS):
            print(nm)
            append_cases(nm, SCENARIOS[nm])
        return
    names = argv or list(SCENARIOS)
    for nm in names:
        print(nm)
        run_case(nm, SCENARIOS[nm])


if __name__ == "__main__":
    main(sys.argv[1:])
