"""Minimal BGZF / BAM / BAI writer for generating golden fixtures (test infrastructure).

Written from the SAM/BAM specification (v1): BGZF members with a 'BC' extra field, the
binary BAM record layout, and the BAI binning + 16 kbp linear index.  The reference's own
reader (bgzf.c / bam.c / bam_index.c under /root/reference) consumes the files this module
writes; `make_golden.py` runs the compiled reference on them to produce the golden TSVs.

Nothing here is product code: the product never writes BAM.
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass, field

BGZF_BLOCK = 0xFF00  # uncompressed bytes per BGZF member (keeps BSIZE < 64 KiB)
EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")

CIGAR_OPS = "MIDNSHP=X"
SEQ_NT16 = {c: i for i, c in enumerate("=ACMGRSVTWYHKDBN")}
# byte -> 4-bit code (upper-cased; anything else -> N = 15), for bytes.translate
_NT16_TR = bytes(SEQ_NT16.get(chr(b).upper(), 15) for b in range(256))


def reg2bin(beg: int, end: int) -> int:
    """SAM spec section 5.3 binning (end exclusive)."""
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def ref_span(cigar: list[tuple[str, int]]) -> int:
    return sum(n for op, n in cigar if op in "MDN=X")


@dataclass
class Read:
    name: str
    tid: int
    pos: int                      # 0-based leftmost
    mapq: int
    flag: int
    cigar: list                   # [(op, len)]
    seq: str                      # query bases (A/C/G/T/N/...)
    qual: list                    # per-base phred ints
    tags: dict = field(default_factory=dict)   # {'RG': 'rg0'} -> Z tags only

    @property
    def end(self) -> int:
        span = ref_span(self.cigar)
        return self.pos + (span if span > 0 else 1)

    def encode(self) -> bytes:
        name = self.name.encode() + b"\0"
        ncig = len(self.cigar)
        cig = b"".join(struct.pack("<I", n << 4 | CIGAR_OPS.index(op)) for op, n in self.cigar)
        lseq = len(self.seq)
        codes = self.seq.encode("latin-1").translate(_NT16_TR) + (b"\0" if lseq & 1 else b"")
        packed = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2))
        qual = bytes(self.qual) if lseq else b""
        aux = b"".join(k.encode() + b"Z" + str(v).encode() + b"\0" for k, v in self.tags.items())
        bin_ = reg2bin(self.pos, self.end)
        core = struct.pack("<iiBBHHHiiii", self.tid, self.pos, len(name), self.mapq, bin_,
                           ncig, self.flag, lseq, -1, -1, 0)
        body = core + name + cig + bytes(packed) + qual + aux
        return struct.pack("<i", len(body)) + body


class BgzfWriter:
    def __init__(self, path: str):
        self.f = open(path, "wb")
        self.buf = bytearray()
        self.coffset = 0  # compressed offset of the block being filled

    def tell(self) -> int:
        """Virtual offset of the next byte written."""
        return (self.coffset << 16) | len(self.buf)

    def write(self, data: bytes) -> None:
        self.buf += data
        while len(self.buf) >= BGZF_BLOCK:
            self._flush(BGZF_BLOCK)

    def _flush(self, n: int) -> None:
        chunk = bytes(self.buf[:n])
        del self.buf[:n]
        comp = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = comp.compress(chunk) + comp.flush()
        bsize = len(cdata) + 25
        hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
        tail = struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
        blk = hdr + cdata + tail
        self.f.write(blk)
        self.coffset += len(blk)

    def flush_block(self) -> None:
        if self.buf:
            self._flush(len(self.buf))

    def close(self) -> None:
        self.flush_block()
        self.f.write(EOF_BLOCK)
        self.f.close()


def write_bam(path: str, header_text: str, refs: list[tuple[str, int]], reads: list[Read]) -> None:
    """Write a coordinate-sorted BAM plus `path + '.bai'`.  `reads` must be sorted by (tid, pos)."""
    w = BgzfWriter(path)
    htxt = header_text.encode()
    hdr = b"BAM\1" + struct.pack("<i", len(htxt)) + htxt + struct.pack("<i", len(refs))
    for name, ln in refs:
        nm = name.encode() + b"\0"
        hdr += struct.pack("<i", len(nm)) + nm + struct.pack("<i", ln)
    w.write(hdr)
    w.flush_block()  # records start on a fresh block (like samtools)

    # per reference: bins -> list of [beg_voff, end_voff]; linear index
    bins = [dict() for _ in refs]
    lin = [dict() for _ in refs]
    last = (-1, -1)
    for r in reads:
        key = (r.tid, r.pos)
        assert key >= last, "reads must be coordinate sorted"
        last = key
        beg_v = w.tell()
        w.write(r.encode())
        end_v = w.tell()
        if r.tid < 0:
            continue
        b = reg2bin(r.pos, r.end)
        chunks = bins[r.tid].setdefault(b, [])
        if chunks and chunks[-1][1] == beg_v:
            chunks[-1][1] = end_v
        else:
            chunks.append([beg_v, end_v])
        for win in range(r.pos >> 14, ((r.end - 1) >> 14) + 1):
            if win not in lin[r.tid] or beg_v < lin[r.tid][win]:
                lin[r.tid][win] = beg_v
    w.close()

    with open(path + ".bai", "wb") as f:
        f.write(b"BAI\1" + struct.pack("<i", len(refs)))
        for t in range(len(refs)):
            f.write(struct.pack("<i", len(bins[t])))
            for b in sorted(bins[t]):
                ch = bins[t][b]
                f.write(struct.pack("<Ii", b, len(ch)))
                for cb, ce in ch:
                    f.write(struct.pack("<QQ", cb, ce))
            n_intv = (max(lin[t]) + 1) if lin[t] else 0
            f.write(struct.pack("<i", n_intv))
            prev = 0
            for i in range(n_intv):
                v = lin[t].get(i, prev)
                prev = v
                f.write(struct.pack("<Q", v))


def write_fasta(path: str, seqs: list[tuple[str, str]], width: int = 60) -> None:
    with open(path, "w") as f:
        for name, s in seqs:
            f.write(f">{name}\n")
            for i in range(0, len(s), width):
                f.write(s[i:i + width] + "\n")
