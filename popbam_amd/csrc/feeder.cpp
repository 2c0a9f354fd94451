// feeder.cpp -- host pileup feeder (include/popbam_feed.h): BGZF/BAM/BAI/FASTA reader and
// the pileup walk that produces the dense batch of the GPU path.
//
// Restates (as behaviour, SAM/BAM spec v1 formats):
//   bgzf.c        blocks of raw-deflate data with a BC extra field, virtual offsets
//                 (block file offset << 16 | offset in the uncompressed block);
//   bam_index.c   bam_fetch (bam_index.c:884-980): reads of `tid` overlapping [beg, end)
//                 (is_overlap, :729-735), in file order, stopping at the first read of
//                 another contig or starting at/after `end`;
//   bam_pileup.c  bam_plp_push / bam_plp_next (:283-407): reads are buffered in push order,
//                 masked by BAM_DEF_MASK, dropped past maxcnt (8000) when they start at the
//                 current pileup position; every position spanned by a buffered read
//                 (bam_calend end, bam.c:20-78) gets a callback with the reads spanning it,
//                 each resolved to a query position / deletion / ref-skip (resolve_cigar2,
//                 :90-235);
//   popbam.cpp    the per-sample partition of call_base (:220-249).
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <memory>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/popbam_feed.h"
#include "pbg_key.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// Compact pieces (pbf_filter.compact, pbg_stream_push_compact): the scan's reference-only test
// (call_kernel.hip call_scan_kernel) on the host -- 1..32 keys, every key's base (bits 0-1) the
// base of an upper-case A/C/G/T reference byte at a called position (bit 7 clear).
inline int ref_base_upper(uint8_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}
inline bool all_on_base(const uint16_t *key, uint32_t n, uint32_t base) {
    uint32_t x = 0;
    for (uint32_t j = 0; j < n; ++j) x |= (key[j] & 3u) ^ base;
    return x == 0;
}

// ---------------------------------------------------------------- raw deflate
// BGZF blocks are raw deflate streams of at most 64 KB.  libdeflate (a system library of this
// image, loaded at run time: its header is not installed) inflates a whole block in one call
// about twice as fast as zlib; zlib's inflate (one reused stream per reader) is the fallback.
struct LibDeflate {
    void *(*alloc)() = nullptr;
    int (*run)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    void (*free_)(void *) = nullptr;
};
const LibDeflate &libdeflate() {
    static LibDeflate ld = [] {
        LibDeflate x;
        if (getenv("POPBAM_NO_LIBDEFLATE")) return x;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return x;
        x.alloc = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        x.run = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_deflate_decompress");
        x.free_ = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        if (!x.alloc || !x.run || !x.free_) x = LibDeflate{};
        return x;
    }();
    return ld;
}
struct Inflater {
    void *ld = nullptr;
    z_stream zs;
    bool zinit = false;
    Inflater() {
        if (libdeflate().alloc) ld = libdeflate().alloc();
    }
    ~Inflater() {
        if (ld) libdeflate().free_(ld);
        if (zinit) inflateEnd(&zs);
    }
    Inflater(const Inflater &) = delete;
    Inflater &operator=(const Inflater &) = delete;
    // true when `in` inflates to exactly `out_n` bytes
    bool run(const uint8_t *in, size_t n, uint8_t *out, size_t out_n) {
        if (ld) {
            size_t got = 0;
            return libdeflate().run(ld, in, n, out, out_n, &got) == 0 && got == out_n;
        }
        if (!zinit) {
            memset(&zs, 0, sizeof(zs));
            if (inflateInit2(&zs, -15) != Z_OK) return false;
            zinit = true;
        } else if (inflateReset(&zs) != Z_OK) {
            return false;
        }
        zs.next_in = const_cast<uint8_t *>(in);
        zs.avail_in = (uInt)n;
        zs.next_out = out;
        zs.avail_out = (uInt)out_n;
        const int r = inflate(&zs, Z_FINISH);
        return r == Z_STREAM_END && zs.avail_out == 0;
    }
};

// ---------------------------------------------------------------- BGZF
struct Bgzf {
    FILE *f = nullptr;
    // uncompressed current block: blk[0, blk_n) (BGZF blocks hold at most 64 KiB; the buffer is
    // never zero-filled, inflate writes every byte)
    std::unique_ptr<uint8_t[]> blk{new uint8_t[65536]};
    size_t blk_n = 0;
    size_t at = 0;                // read position in blk
    uint64_t blk_addr = 0;        // file offset of the current block
    uint64_t next_addr = 0;       // file offset of the next block
    uint64_t fpos = ~0ull;        // the FILE's position (a block after the previous one needs no seek)
    std::vector<uint8_t> cbuf;
    Inflater inf;
    double t_inflate = 0.0;       // seconds in inflate
    uint64_t n_blocks = 0, bytes_in = 0, bytes_out = 0;

    ~Bgzf() {
        if (f) fclose(f);
    }
    // loads the block at file offset `addr`; false at EOF, throws nothing
    int load(uint64_t addr) {
        if (addr != fpos && fseeko(f, (off_t)addr, SEEK_SET) != 0) return fail(PBF_E_IO, "seek failed");
        fpos = ~0ull;
        uint8_t h[18];
        size_t got = fread(h, 1, 18, f);
        blk_n = 0;
        at = 0;
        blk_addr = addr;
        if (got == 0) {
            next_addr = addr;
            return 0;   // EOF
        }
        if (got < 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4))
            return fail(PBF_E_FORMAT, "not a BGZF block");
        const int xlen = h[10] | h[11] << 8;
        uint8_t extra[65536 + 6];
        memcpy(extra, h + 12, std::min(xlen, 6));
        if (xlen > 6 && fread(extra + 6, 1, xlen - 6, f) != (size_t)(xlen - 6))
            return fail(PBF_E_FORMAT, "truncated BGZF header");
        int bsize = -1;
        for (int p = 0; p + 4 <= xlen;) {
            const int slen = extra[p + 2] | extra[p + 3] << 8;
            if (extra[p] == 'B' && extra[p + 1] == 'C' && slen == 2) bsize = extra[p + 4] | extra[p + 5] << 8;
            p += 4 + slen;
        }
        if (bsize < 0) return fail(PBF_E_FORMAT, "BGZF block without BC field");
        const int cdata = bsize - xlen - 19;
        if (cdata < 0) return fail(PBF_E_FORMAT, "bad BGZF block size");
        cbuf.resize((size_t)cdata + 8);
        // the 6 bytes of extra already read overlap the data when xlen < 6 (never for BGZF)
        if (fread(cbuf.data(), 1, (size_t)cdata + 8, f) != (size_t)cdata + 8)
            return fail(PBF_E_FORMAT, "truncated BGZF block");
        const uint32_t isize = cbuf[cdata + 4] | cbuf[cdata + 5] << 8 | cbuf[cdata + 6] << 16 |
                               (uint32_t)cbuf[cdata + 7] << 24;
        if (isize > 65536) return fail(PBF_E_FORMAT, "BGZF block larger than 64 KiB");
        blk_n = isize;
        next_addr = addr + (uint64_t)bsize + 1;
        fpos = next_addr;
        if (isize == 0) return 1;
        const auto t0 = Clock::now();
        const bool ok = inf.run(cbuf.data(), (size_t)cdata, blk.get(), isize);
        t_inflate += secs(t0, Clock::now());
        ++n_blocks;
        bytes_in += (uint64_t)cdata;
        bytes_out += isize;
        if (!ok) return fail(PBF_E_FORMAT, "corrupt BGZF block");
        return 1;
    }
    int seek(uint64_t voff) {
        const int r = load(voff >> 16);
        if (r < 0) return r;
        at = (size_t)(voff & 0xFFFF);
        return 0;
    }
    // reads n bytes; returns bytes read (< n only at EOF) or a negative error
    long read(void *dst, size_t n) {
        uint8_t *o = (uint8_t *)dst;
        size_t done = 0;
        while (done < n) {
            if (at >= blk_n) {
                const int r = load(next_addr);
                if (r < 0) return r;
                if (r == 0) break;
                continue;
            }
            const size_t k = std::min(n - done, blk_n - at);
            memcpy(o + done, blk.get() + at, k);
            at += k;
            done += k;
        }
        return (long)done;
    }
    // the next n bytes in place when the current block holds them (the next block is loaded when
    // the current one is used up); nullptr otherwise (read() then copies across the boundary).
    // `eof` is set when no byte is left at all.
    const uint8_t *peek(size_t n, bool &eof, int &err) {
        eof = false;
        err = 0;
        while (at >= blk_n) {
            const int r = load(next_addr);
            if (r < 0) {
                err = r;
                return nullptr;
            }
            if (r == 0) {
                eof = true;
                return nullptr;
            }
        }
        return at + n <= blk_n ? blk.get() + at : nullptr;
    }
    void skip(size_t n) { at += n; }
};

// ---------------------------------------------------------------- BAM records
struct Rec {
    int32_t tid, pos, end;        // end = bam_calend
    uint16_t flag;
    uint8_t mapq;
    std::vector<uint32_t> cigar;
    std::vector<uint8_t> nt16, qual;
    std::string rg;
    bool has_rg;
};

uint32_t le32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

// size of one aux value of type t at p (0 = unknown / malformed)
size_t aux_size(char t, const uint8_t *p, const uint8_t *e) {
    switch (t) {
        case 'A': case 'c': case 'C': return 1;
        case 's': case 'S': return 2;
        case 'i': case 'I': case 'f': return 4;
        case 'd': return 8;
        case 'Z': case 'H': {
            const uint8_t *q = p;
            while (q < e && *q) ++q;
            return q < e ? (size_t)(q - p) + 1 : 0;
        }
        case 'B': {
            if (e - p < 5) return 0;
            const char st = (char)p[0];
            const uint32_t n = le32(p + 1);
            const size_t es = aux_size(st, p, e);
            if (!es || st == 'Z' || st == 'H' || st == 'B') return 0;
            return 5 + (size_t)n * es;
        }
        default: return 0;
    }
}

int32_t calend(int32_t pos, const std::vector<uint32_t> &cig) {
    int32_t end = pos;
    for (uint32_t c : cig) {
        const uint32_t op = c & 0xF;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) end += (int32_t)(c >> 4);   // M D N = X
    }
    return end;
}

// bam_read1: 1 = record, 0 = EOF, < 0 error
int read_rec(Bgzf &z, Rec &r) {
    uint8_t b4[4];
    const long g = z.read(b4, 4);
    if (g == 0) return 0;
    if (g != 4) return fail(PBF_E_FORMAT, "truncated BAM record");
    const uint32_t bs = le32(b4);
    if (bs < 32) return fail(PBF_E_FORMAT, "bad BAM record size");
    std::vector<uint8_t> buf(bs);
    if (z.read(buf.data(), bs) != (long)bs) return fail(PBF_E_FORMAT, "truncated BAM record");
    const uint8_t *p = buf.data(), *e = p + bs;
    r.tid = (int32_t)le32(p);
    r.pos = (int32_t)le32(p + 4);
    const uint32_t bin_mq_nl = le32(p + 8), flag_nc = le32(p + 12);
    const int32_t l_seq = (int32_t)le32(p + 16);
    const int l_name = bin_mq_nl & 0xFF;
    r.mapq = (uint8_t)((bin_mq_nl >> 8) & 0xFF);
    r.flag = (uint16_t)(flag_nc >> 16);
    const int n_cig = flag_nc & 0xFFFF;
    const uint8_t *q = p + 32 + l_name;
    if (l_seq < 0 || q + 4 * (size_t)n_cig + (l_seq + 1) / 2 + l_seq > e)
        return fail(PBF_E_FORMAT, "BAM record fields exceed its size");
    r.cigar.resize(n_cig);
    for (int i = 0; i < n_cig; ++i) r.cigar[i] = le32(q + 4 * i);
    q += 4 * (size_t)n_cig;
    r.nt16.resize(l_seq);
    for (int i = 0; i < l_seq; ++i) r.nt16[i] = (i & 1) ? (q[i >> 1] & 0xF) : (q[i >> 1] >> 4);
    q += (l_seq + 1) / 2;
    r.qual.assign(q, q + l_seq);
    q += l_seq;
    r.has_rg = false;
    while (q + 3 <= e) {   // bam_aux_get(b, "RG")
        const char t = (char)q[2];
        const size_t sz = aux_size(t, q + 3, e);
        if (!sz) break;
        if (q[0] == 'R' && q[1] == 'G') {
            r.has_rg = true;
            if (t == 'Z' || t == 'H') r.rg.assign((const char *)q + 3);
            else r.rg.clear();   // non-string RG: the reference passes its raw bytes as a key
            break;
        }
        q += 3 + sz;
    }
    r.end = n_cig ? calend(r.pos, r.cigar) : r.pos;
    return 1;
}

struct Chunk {
    uint64_t beg, end;
};

}  // namespace

struct pbf_bam {
    Bgzf z;
    std::string text;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    uint64_t first_rec = 0;   // virtual offset of the first record
    bool has_index = false;
    std::vector<std::unordered_map<uint32_t, std::vector<Chunk>>> bins;   // per tid
    std::vector<std::vector<uint64_t>> linear;                              // per tid
};

namespace {

int load_index(pbf_bam *b, const std::string &path) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return 0;
    std::vector<uint8_t> d;
    {
        uint8_t tmp[1 << 16];
        size_t k;
        while ((k = fread(tmp, 1, sizeof(tmp), f)) > 0) d.insert(d.end(), tmp, tmp + k);
        fclose(f);
    }
    size_t p = 0;
    auto need = [&](size_t n) { return p + n <= d.size(); };
    if (!need(8) || memcmp(d.data(), "BAI\1", 4) != 0) return fail(PBF_E_FORMAT, "bad BAI magic");
    p = 4;
    const int32_t n_ref = (int32_t)le32(&d[p]);
    p += 4;
    b->bins.assign(n_ref, {});
    b->linear.assign(n_ref, {});
    auto u64 = [&](size_t o) { return (uint64_t)le32(&d[o]) | (uint64_t)le32(&d[o + 4]) << 32; };
    for (int32_t t = 0; t < n_ref; ++t) {
        if (!need(4)) return fail(PBF_E_FORMAT, "truncated BAI");
        const int32_t n_bin = (int32_t)le32(&d[p]);
        p += 4;
        for (int32_t i = 0; i < n_bin; ++i) {
            if (!need(8)) return fail(PBF_E_FORMAT, "truncated BAI");
            const uint32_t bin = le32(&d[p]);
            const int32_t n_chunk = (int32_t)le32(&d[p + 4]);
            p += 8;
            if (!need(16 * (size_t)n_chunk)) return fail(PBF_E_FORMAT, "truncated BAI");
            auto &v = b->bins[t][bin];
            for (int32_t c = 0; c < n_chunk; ++c, p += 16) v.push_back({u64(p), u64(p + 8)});
        }
        if (!need(4)) return fail(PBF_E_FORMAT, "truncated BAI");
        const int32_t n_intv = (int32_t)le32(&d[p]);
        p += 4;
        if (!need(8 * (size_t)n_intv)) return fail(PBF_E_FORMAT, "truncated BAI");
        for (int32_t i = 0; i < n_intv; ++i, p += 8) b->linear[t].push_back(u64(p));
    }
    b->has_index = true;
    return 0;
}

// bins overlapping [beg, end) (SAM spec §5.3 reg2bins)
void reg2bins(int32_t beg, int32_t end, std::vector<uint32_t> &out) {
    out.clear();
    --end;
    out.push_back(0);
    const int shifts[5] = {26, 23, 20, 17, 14};
    const uint32_t offs[5] = {1, 9, 73, 585, 4681};
    for (int l = 0; l < 5; ++l)
        for (uint32_t k = offs[l] + (uint32_t)(beg >> shifts[l]); k <= offs[l] + (uint32_t)(end >> shifts[l]); ++k)
            out.push_back(k);
}

// start virtual offset for reads of tid overlapping [beg, end); false if none can exist
bool region_start(const pbf_bam *b, int tid, int32_t beg, int32_t end, uint64_t &start) {
    if (!b->has_index || tid >= (int)b->bins.size()) {
        start = b->first_rec;
        return true;
    }
    const auto &lin = b->linear[tid];
    uint64_t min_off = 0;
    if (!lin.empty()) {
        size_t i = std::min<size_t>((size_t)(beg >> 14), lin.size() - 1);
        while (i > 0 && lin[i] == 0) --i;
        min_off = lin[i];
    }
    std::vector<uint32_t> bl;
    reg2bins(beg, end, bl);
    bool any = false;
    uint64_t best = ~0ULL;
    for (uint32_t bin : bl) {
        auto it = b->bins[tid].find(bin);
        if (it == b->bins[tid].end()) continue;
        for (const Chunk &c : it->second)
            if (c.end > min_off) {
                best = std::min(best, std::max(c.beg, min_off));
                any = true;
            }
    }
    start = best;
    return any;
}

// one buffered read of the pileup (bam_plp node) with its CIGAR walk state
struct Node {
    const Rec *r;
    int k = -1;          // current CIGAR op (resolve_cigar2 cstate: k, x = ref pos, y = query pos)
    int32_t x = 0, y = 0;
};

// resolve_cigar2 outcome at `pos` (pos in [beg, end)): 0 base at *qpos, 1 deletion, 2 ref skip
int resolve(Node &n, int32_t pos, int32_t *qpos) {
    const std::vector<uint32_t> &cg = n.r->cigar;
    const int nc = (int)cg.size();
    if (n.k < 0) {   // first visit: skip to the first M / D / = / X, accumulating N / I / S
        n.x = n.r->pos;
        n.y = 0;
        int k = 0;
        for (; k < nc; ++k) {
            const uint32_t op = cg[k] & 0xF, l = cg[k] >> 4;
            if (op == 0 || op == 2 || op == 7 || op == 8) break;
            if (op == 3) n.x += (int32_t)l;
            else if (op == 1 || op == 4) n.y += (int32_t)l;
        }
        n.k = k < nc ? k : nc - 1;
    }
    // advance to the op containing pos
    for (;;) {
        const uint32_t op = cg[n.k] & 0xF, l = cg[n.k] >> 4;
        const bool cons_ref = op == 0 || op == 2 || op == 3 || op == 7 || op == 8;
        if (cons_ref && pos - n.x < (int32_t)l) break;
        if (n.k + 1 >= nc) break;
        if (op == 0 || op == 7 || op == 8 || op == 1 || op == 4) n.y += (int32_t)l;
        if (cons_ref) n.x += (int32_t)l;
        ++n.k;
    }
    const uint32_t op = cg[n.k] & 0xF;
    if (op == 2) return 1;
    if (op == 3) return 2;
    *qpos = n.y + (pos - n.x);
    return 0;
}

}  // namespace

extern "C" {

const char *pbf_last_error(void) { return g_err.c_str(); }

int pbf_open(pbf_bam **out, const char *path) {
    if (!out || !path) return fail(PBF_E_ARG, "null argument");
    *out = nullptr;
    pbf_bam *b = new pbf_bam();
    b->z.f = fopen(path, "rb");
    if (!b->z.f) {
        delete b;
        return fail(PBF_E_IO, std::string("cannot open ") + path);
    }
    setvbuf(b->z.f, nullptr, _IOFBF, 1 << 20);
    int r = b->z.load(0);
    if (r <= 0) {
        delete b;
        return r < 0 ? r : fail(PBF_E_FORMAT, "empty BAM file");
    }
    uint8_t m[8];
    if (b->z.read(m, 8) != 8 || memcmp(m, "BAM\1", 4) != 0) {
        delete b;
        return fail(PBF_E_FORMAT, "not a BAM file");
    }
    const uint32_t l_text = le32(m + 4);
    b->text.resize(l_text);
    if (l_text && b->z.read(&b->text[0], l_text) != (long)l_text) {
        delete b;
        return fail(PBF_E_FORMAT, "truncated BAM header");
    }
    b->text = std::string(b->text.c_str());   // header text up to its first NUL
    uint8_t n4[4];
    if (b->z.read(n4, 4) != 4) {
        delete b;
        return fail(PBF_E_FORMAT, "truncated BAM header");
    }
    const int32_t n_ref = (int32_t)le32(n4);
    for (int32_t i = 0; i < n_ref; ++i) {
        if (b->z.read(n4, 4) != 4) {
            delete b;
            return fail(PBF_E_FORMAT, "truncated reference list");
        }
        const uint32_t ln = le32(n4);
        std::string nm(ln, '\0');
        if (b->z.read(&nm[0], ln) != (long)ln || b->z.read(n4, 4) != 4) {
            delete b;
            return fail(PBF_E_FORMAT, "truncated reference list");
        }
        b->names.push_back(std::string(nm.c_str()));
        b->lens.push_back((int64_t)le32(n4));
    }
    b->first_rec = b->z.blk_addr << 16 | b->z.at;
    if ((r = load_index(b, std::string(path) + ".bai")) < 0) {
        delete b;
        return r;
    }
    *out = b;
    return PBF_OK;
}

void pbf_close(pbf_bam *b) { delete b; }
const char *pbf_header_text(const pbf_bam *b) { return b ? b->text.c_str() : ""; }
int pbf_n_refs(const pbf_bam *b) { return b ? (int)b->names.size() : 0; }
const char *pbf_ref_name(const pbf_bam *b, int tid) {
    return b && tid >= 0 && tid < (int)b->names.size() ? b->names[tid].c_str() : nullptr;
}
int64_t pbf_ref_len(const pbf_bam *b, int tid) {
    return b && tid >= 0 && tid < (int)b->lens.size() ? b->lens[tid] : -1;
}
int pbf_has_index(const pbf_bam *b) { return b && b->has_index ? 1 : 0; }

void pbf_batch_free(pbf_batch *o) {
    if (!o) return;
    free(o->ref);
    free(o->depth);
    free(o->block_off);
    free(o->reads);
    memset(o, 0, sizeof(*o));
}

void pbf_free(void *p) { free(p); }

}  // extern "C"

namespace {

// bam_fetch: reads of `tid` overlapping [lo, hi) in file order (bam_index.c:884-980)
int fetch_region(pbf_bam *b, int tid, int32_t lo, int32_t hi, std::vector<Rec> &recs) {
    recs.clear();
    uint64_t start;
    if (hi <= lo || !region_start(b, tid, lo, hi, start)) return PBF_OK;
    int r = b->z.seek(start);
    if (r < 0) return r;
    Rec rec;
    while ((r = read_rec(b->z, rec)) == 1) {
        if (rec.tid != tid) {
            if (b->has_index || (rec.tid > tid)) break;   // sorted: past the contig
            continue;
        }
        if (rec.pos >= hi) break;
        const int32_t oend = rec.cigar.empty() ? rec.pos + 1 : rec.end;
        if (oend > lo && rec.pos < hi) recs.push_back(rec);
    }
    return r < 0 ? r : PBF_OK;
}

constexpr int kMaxCnt = 8000;                               // bam_plp maxcnt (bam_pileup.c:375)
constexpr uint16_t kDefMask = 0x4 | 0x100 | 0x200 | 0x400;   // BAM_DEF_MASK (bam.h:123)

struct WalkCfg {
    std::unordered_map<std::string, int32_t> rgmap;
    int32_t fallback;
    int ns, max_depth;
};

// positions [p0, p0 + n) of a batch, filled in position order by one or more walks
struct WalkOut {
    int32_t p0;
    uint32_t n;
    uint8_t *ref;
    uint16_t *depth;
    std::vector<uint32_t> reads;
};

// One bam_plp walk (bam_plp_push / bam_plp_next) over `recs`; positions in [ebeg, eend) get
// the callback's per-sample partition (popbam.cpp:220-249) written into `o`.  Walks that fill
// one batch must come in increasing, disjoint [ebeg, eend).
int walk(const std::vector<Rec> &recs, int32_t ebeg, int32_t eend, const WalkCfg &cf, WalkOut &o) {
    std::vector<Node> buf;            // push order
    std::vector<std::vector<uint32_t>> per(cf.ns);
    int32_t ipos = 0, itid = 0, max_pos = -1, max_tid = -1;
    int err = 0;
    auto emit = [&](int32_t pos) {
        if (pos < ebeg || pos >= eend) return;
        const uint32_t i = (uint32_t)(pos - o.p0);
        o.ref[i] &= 0x7F;
        for (auto &v : per) v.clear();
        for (Node &n : buf) {
            if (n.r->pos > pos || n.r->end <= pos) continue;
            int32_t qp = 0;
            const int kind = resolve(n, pos, &qp);
            if (kind != 0 || (n.r->flag & 0x4)) continue;
            if (!n.r->has_rg) continue;
            auto it = cf.rgmap.find(n.r->rg);
            const int32_t s = it != cf.rgmap.end() ? it->second : cf.fallback;
            if (s < 0 || s >= cf.ns) {
                if (!err) err = fail(PBF_E_RG, "Problem assigning read group " + n.r->rg +
                                                   " to a sample.\nPlease check BAM header for correct SM and PO tags");
                continue;
            }
            if ((int)per[s].size() >= cf.max_depth) continue;
            const uint32_t strand = (n.r->flag >> 4) & 1u;
            per[s].push_back((uint32_t)n.r->qual[qp] | (uint32_t)n.r->mapq << 8 | (uint32_t)n.r->nt16[qp] << 16 |
                             strand << 20);
        }
        for (int s = 0; s < cf.ns; ++s) {
            o.depth[(size_t)i * cf.ns + s] = (uint16_t)per[s].size();
            o.reads.insert(o.reads.end(), per[s].begin(), per[s].end());
        }
    };
    // emits every pending position below max_pos (or all at EOF), dropping finished reads
    auto next = [&](bool eof) {
        while (eof || max_tid > itid || (max_tid == itid && max_pos > ipos)) {
            bool any = false;
            size_t w = 0;
            for (size_t j = 0; j < buf.size(); ++j) {
                Node &n = buf[j];
                if (n.r->tid < itid || (n.r->tid == itid && n.r->end <= ipos)) continue;   // removed
                if (n.r->tid == itid && n.r->pos <= ipos) any = true;
                buf[w++] = n;
            }
            buf.resize(w);
            if (any) emit(ipos);
            if (!buf.empty()) {
                const Rec *h = buf.front().r;
                if (itid < h->tid) {
                    itid = h->tid;
                    ipos = h->pos;
                } else if (ipos < h->pos) {
                    ipos = h->pos;
                } else {
                    ++ipos;
                }
            } else {
                if (eof) break;
                ++ipos;   // empty buffer: the reference steps through the gap one position at a time
                if (max_pos > ipos) ipos = max_pos;   // (no callbacks there; skip ahead)
            }
        }
    };
    for (const Rec &r : recs) {
        if (r.tid < 0 || (r.flag & kDefMask)) continue;
        if (itid == r.tid && ipos == r.pos && (int)buf.size() + 2 > kMaxCnt) continue;   // maxcnt
        max_tid = r.tid;
        max_pos = r.pos;
        if (r.end > ipos || r.tid > itid) {
            Node n;
            n.r = &r;
            buf.push_back(n);
        }
        next(false);
    }
    next(true);
    return err;
}

// Upper bound of the pileup buffer at each maxcnt test: a read starting at p meets at most
// the unmasked reads before it that still reach p (the walk drops a read only after passing
// its end).  Returns the largest bound over the reads that matter for positions >= from
// (reads starting there, or reaching it).
int max_buffer_bound(const std::vector<Rec> &a, int32_t from) {
    std::vector<int32_t> ends;   // min-heap of the ends of earlier reads
    int best = 0;
    for (const Rec &r : a) {
        if (r.tid < 0 || (r.flag & kDefMask)) continue;
        while (!ends.empty() && ends.front() < r.pos) {
            std::pop_heap(ends.begin(), ends.end(), std::greater<int32_t>());
            ends.pop_back();
        }
        if (r.pos >= from || r.end >= from) best = std::max(best, (int)ends.size());
        ends.push_back(std::max(r.end, r.pos + 1));
        std::push_heap(ends.begin(), ends.end(), std::greater<int32_t>());
    }
    return best;
}

// Positions [cb, ce) of a region [rbeg, rend) that the reference walks window by window
// (win > 0: window k is [rbeg + k*win, rbeg + (k+1)*win - 1), a fresh bam_fetch + pileup per
// window, pop_nucdiv.cpp:57-125; win == 0: one walk of the whole region).
// When no read that reaches [cb, ce) can meet a full buffer (max_buffer_bound + 2 <= maxcnt),
// every walk keeps every read, so one walk of the reads overlapping [cb, ce) gives the
// reference's pileup there.  Otherwise the maxcnt drops depend on where the reference's walk
// started: walk each window of the reference (and each position between windows) on its own.
int chunk_walk(pbf_bam *b, int tid, int32_t cb, int32_t ce, int32_t rbeg, int32_t rend, int32_t win,
               const WalkCfg &cf, WalkOut &o) {
    std::vector<Rec> recs, early;
    int r = fetch_region(b, tid, std::max(0, cb - 1), ce, recs);
    if (r != PBF_OK) return r;
    int32_t lo = cb;
    for (const Rec &x : recs)
        if (!(x.flag & kDefMask)) lo = std::min(lo, x.pos);
    int bound;
    if (lo < cb) {   // the reads before cb that reach it: their tests see reads ending before cb too
        r = fetch_region(b, tid, std::max(0, lo - 1), cb, early);
        if (r != PBF_OK) return r;
        std::vector<Rec> all;
        for (const Rec &x : early)
            if (x.pos < cb) all.push_back(x);
        for (const Rec &x : recs)
            if (x.pos >= cb) all.push_back(x);
        bound = max_buffer_bound(all, cb);
    } else {
        bound = max_buffer_bound(recs, cb);
    }
    if (bound + 2 <= kMaxCnt) return walk(recs, cb, ce, cf, o);
    // crowded: the reference's own walks
    int32_t a = cb;
    while (a < ce) {
        int32_t sa, sb;   // the reference walk that covers position a
        if (win <= 0) {
            sa = rbeg, sb = rend;
        } else {
            const int64_t k = ((int64_t)a - rbeg) / win;
            const int64_t wb = rbeg + k * win, we = wb + win - 1;
            if (a < we) sa = (int32_t)wb, sb = (int32_t)std::min<int64_t>(we, rend);
            else sa = a, sb = a + 1;   // the last base of a window: in no window
        }
        sb = std::max(sb, a + 1);
        r = fetch_region(b, tid, sa, sb, recs);
        if (r != PBF_OK) return r;
        const int32_t e = std::min(sb, ce);
        r = walk(recs, a, e, cf, o);
        if (r != PBF_OK) return r;
        a = e;
    }
    return PBF_OK;
}

int batch_alloc(pbf_batch *out, int32_t beg, uint32_t L, int ns, const char *refseq) {
    memset(out, 0, sizeof(*out));
    out->n_sites = L;
    out->pos0 = beg;
    out->ref = (uint8_t *)malloc(std::max<size_t>(L, 1));
    out->depth = (uint16_t *)calloc(std::max<size_t>((size_t)L * ns, 1), sizeof(uint16_t));
    out->block_off = (uint64_t *)calloc(L / 64 + 2, sizeof(uint64_t));
    if (!out->ref || !out->depth || !out->block_off) {
        pbf_batch_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    for (uint32_t i = 0; i < L; ++i) out->ref[i] = (uint8_t)refseq[beg + i] | 0x80;
    return PBF_OK;
}

// block offsets + reads of a filled batch
int batch_finish(pbf_batch *out, int ns, std::vector<uint32_t> &reads) {
    const uint32_t L = out->n_sites;
    uint64_t acc = 0;
    for (uint32_t bk = 0; bk * 64 < L; ++bk) {
        out->block_off[bk] = acc;
        const uint32_t hi = std::min(L, bk * 64 + 64);
        for (uint32_t i = bk * 64; i < hi; ++i)
            for (int s = 0; s < ns; ++s) acc += out->depth[(size_t)i * ns + s];
    }
    out->block_off[(L + 63) / 64] = acc;
    out->n_reads = reads.size();
    out->reads = (uint32_t *)malloc(std::max<size_t>(reads.size(), 1) * sizeof(uint32_t));
    if (!out->reads) {
        pbf_batch_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    if (!reads.empty()) memcpy(out->reads, reads.data(), reads.size() * sizeof(uint32_t));
    return PBF_OK;
}

WalkCfg make_cfg(const char *const *rg_ids, const int32_t *rg_sample, int n_rg, int32_t fallback, int ns,
                 int max_depth) {
    WalkCfg cf;
    for (int i = 0; i < n_rg; ++i) cf.rgmap[rg_ids[i]] = rg_sample[i];
    cf.fallback = fallback;
    cf.ns = ns;
    cf.max_depth = max_depth;
    return cf;
}

// one piece [cb, ce) of a region as a raw batch
int piece_batch(pbf_bam *b, int tid, int32_t cb, int32_t ce, int32_t rbeg, int32_t rend, int32_t win,
                const char *refseq, const WalkCfg &cf, pbf_batch *out) {
    int r = batch_alloc(out, cb, (uint32_t)(ce - cb), cf.ns, refseq);
    if (r != PBF_OK) return r;
    WalkOut o{cb, (uint32_t)(ce - cb), out->ref, out->depth, {}};
    r = chunk_walk(b, tid, cb, ce, rbeg, rend, win, cf, o);
    if (r != PBF_OK) {
        pbf_batch_free(out);
        return r;
    }
    return batch_finish(out, cf.ns, o.reads);
}


// ---------------------------------------------------------------- key batches, fast path
// The key batch of a piece straight from the records: no per-record heap objects (records are
// parsed into one arena per piece), the read group resolved to a sample once per record (the
// reference's bam_aux_get + khash lookup per read per position, popbam.cpp:222-237), and the
// pileup walked with the reads that span each position kept in push (file) order -- the
// buffer bam_plp_push / bam_plp_next keep (bam_pileup.c:283-407) whenever no read meets a full
// buffer (maxcnt), which pieces where one can fall back to the window-by-window walk above.

struct Rec2 {
    int32_t tid, pos, end;   // end = bam_calend
    uint16_t flag, n_cigar;
    uint8_t mapq, strand;
    int32_t l_seq;
    int32_t sample;          // >= 0; -1 no RG (skipped); -2 RG not assigned to a sample
    size_t off;              // arena: cigar (n_cigar u32), packed seq ((l_seq + 1) / 2), qual (l_seq), RG (NUL-terminated)
};
struct Arena {   // grows without zero-filling (every byte is written before it is read)
    uint8_t *p = nullptr;
    size_t n = 0, cap = 0;
    ~Arena() { free(p); }
    uint8_t *grow(size_t k) {
        if (n + k > cap) {
            const size_t nc = std::max(n + k, cap * 2 + (1 << 20));
            uint8_t *q = (uint8_t *)realloc(p, nc);
            if (!q) return nullptr;
            p = q;
            cap = nc;
        }
        uint8_t *at = p + n;
        n += k;
        return at;
    }
    const uint8_t *data() const { return p; }
    size_t size() const { return n; }
};
struct RecSet {
    std::vector<Rec2> r;
    Arena arena;
    std::vector<uint8_t> scratch;
    void clear() {
        r.clear();
        arena.n = 0;
    }
};

// the sample of a read group (the callback's partition, popbam.cpp:222-237), looked up without
// copying the tag (views into the WalkCfg's keys, which outlive the index)
struct RgIndex {
    // open addressing over (length, first 8 bytes): one probe and one compare for the few read
    // groups of a BAM (a std::unordered_map's string hash cost ~1/3 of a record's decode)
    struct Slot {
        const char *name = nullptr;
        uint32_t len = 0;
        int32_t sample = 0;
    };
    std::vector<Slot> t;
    uint32_t mask = 0;
    int32_t fallback;
    int ns;
    static uint32_t hash(const char *s, size_t len) {
        uint64_t w = 0;
        memcpy(&w, s, std::min<size_t>(len, 8));
        w ^= (uint64_t)len * 0x9E3779B97F4A7C15ull;
        w *= 0xBF58476D1CE4E5B9ull;
        return (uint32_t)(w >> 32);
    }
    explicit RgIndex(const WalkCfg &cf) : fallback(cf.fallback), ns(cf.ns) {
        size_t cap = 16;
        while (cap < 4 * cf.rgmap.size()) cap *= 2;
        t.resize(cap);
        mask = (uint32_t)cap - 1;
        for (const auto &kv : cf.rgmap) {
            uint32_t h = hash(kv.first.data(), kv.first.size()) & mask;
            while (t[h].name && !(t[h].len == kv.first.size() && memcmp(t[h].name, kv.first.data(), t[h].len) == 0))
                h = (h + 1) & mask;
            t[h] = Slot{kv.first.data(), (uint32_t)kv.first.size(), kv.second};
        }
    }
    int32_t sample_of(const char *rg, bool has_rg) const {
        if (!has_rg) return -1;
        const size_t len = strlen(rg);
        int32_t s = fallback;
        for (uint32_t h = hash(rg, len) & mask; t[h].name; h = (h + 1) & mask)
            if (t[h].len == len && memcmp(t[h].name, rg, len) == 0) {
                s = t[h].sample;
                break;
            }
        return (s < 0 || s >= ns) ? -2 : s;
    }
};

// bam_read1 into the arena: 1 = record (kept when of `tid` and overlapping [lo, hi)), 0 = EOF,
// 2 = past the region (stop), < 0 error
int read_rec2(Bgzf &z, RecSet &rs, int tid, int32_t lo, int32_t hi, bool has_index, const RgIndex &cf) {
    // the record in place when it lies inside the current block (most do), else copied out
    bool eof = false;
    int err = 0;
    const uint8_t *p = nullptr;
    uint32_t bs = 0;
    if (const uint8_t *h = z.peek(4, eof, err)) {
        bs = le32(h);
        if (bs >= 32 && (p = z.peek(4 + (size_t)bs, eof, err)) != nullptr) {
            p += 4;
            z.skip(4 + (size_t)bs);
        }
    }
    if (err) return err;
    if (!p) {
        if (eof) return 0;
        uint8_t b4[4];
        const long g = z.read(b4, 4);
        if (g == 0) return 0;
        if (g != 4) return fail(PBF_E_FORMAT, "truncated BAM record");
        bs = le32(b4);
        if (bs < 32) return fail(PBF_E_FORMAT, "bad BAM record size");
        if (rs.scratch.size() < bs) rs.scratch.resize(bs);
        if (z.read(rs.scratch.data(), bs) != (long)bs) return fail(PBF_E_FORMAT, "truncated BAM record");
        p = rs.scratch.data();
    }
    const uint8_t *e = p + bs;
    Rec2 r;
    r.tid = (int32_t)le32(p);
    r.pos = (int32_t)le32(p + 4);
    if (r.tid != tid) return (has_index || r.tid > tid) ? 2 : 1;   // sorted: past the contig (or skip)
    if (r.pos >= hi) return 2;
    const uint32_t bin_mq_nl = le32(p + 8), flag_nc = le32(p + 12);
    const int32_t l_seq = (int32_t)le32(p + 16);
    const int l_name = bin_mq_nl & 0xFF;
    r.mapq = (uint8_t)((bin_mq_nl >> 8) & 0xFF);
    r.flag = (uint16_t)(flag_nc >> 16);
    r.strand = (uint8_t)((r.flag >> 4) & 1u);
    const int n_cig = flag_nc & 0xFFFF;
    const uint8_t *q = p + 32 + l_name;
    if (l_seq < 0 || q + 4 * (size_t)n_cig + (l_seq + 1) / 2 + l_seq > e)
        return fail(PBF_E_FORMAT, "BAM record fields exceed its size");
    int32_t end = r.pos;
    for (int i = 0; i < n_cig; ++i) {
        const uint32_t c = le32(q + 4 * i), op = c & 0xF;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) end += (int32_t)(c >> 4);
    }
    r.end = end;
    const int32_t oend = n_cig ? end : r.pos + 1;
    if (!(oend > lo && r.pos < hi)) return 1;   // not overlapping (is_overlap, bam_index.c:729-735)
    r.n_cigar = (uint16_t)n_cig;
    r.l_seq = l_seq;
    const uint8_t *aux = q + 4 * (size_t)n_cig + (l_seq + 1) / 2 + l_seq;
    const char *rg = nullptr;
    bool has_rg = false;
    for (const uint8_t *a = aux; a + 3 <= e;) {   // bam_aux_get(b, "RG")
        const char t = (char)a[2];
        const size_t sz = aux_size(t, a + 3, e);
        if (!sz) break;
        if (a[0] == 'R' && a[1] == 'G') {
            has_rg = true;
            rg = (t == 'Z' || t == 'H') ? (const char *)a + 3 : "";   // non-string RG: its raw bytes (feeder.cpp Rec)
            break;
        }
        a += 3 + sz;
    }
    r.sample = cf.sample_of(rg ? rg : "", has_rg);
    const size_t rglen = r.sample == -2 ? strlen(rg) + 1 : 0;   // kept for the error message only
    const size_t need = 4 * (size_t)n_cig + (l_seq + 1) / 2 + l_seq + rglen;
    r.off = rs.arena.size();
    uint8_t *dst = rs.arena.grow(need);
    if (!dst) return fail(PBF_E_IO, "out of host memory");
    memcpy(dst, q, need - rglen);
    if (rglen) memcpy(dst + need - rglen, rg, rglen);
    rs.r.push_back(r);
    return 1;
}

// bam_fetch into the arena: reads of `tid` overlapping [lo, hi) in file order
int fetch2(pbf_bam *b, int tid, int32_t lo, int32_t hi, const RgIndex &cf, RecSet &rs) {
    rs.clear();
    uint64_t start;
    if (hi <= lo || !region_start(b, tid, lo, hi, start)) return PBF_OK;
    int r = b->z.seek(start);
    if (r < 0) return r;
    while ((r = read_rec2(b->z, rs, tid, lo, hi, b->has_index, cf)) == 1) {
    }
    return r < 0 ? r : PBF_OK;
}

// resolve_cigar2 (bam_pileup.c:90-235) on a Rec2, the cursor kept in (k, x, y) as Node does
struct Cur {
    const Rec2 *r;
    int k;
    int32_t x, y;
};
inline int resolve2(Cur &n, const uint32_t *cg, int32_t pos, int32_t *qpos) {
    const int nc = n.r->n_cigar;
    if (n.k < 0) {
        n.x = n.r->pos;
        n.y = 0;
        int k = 0;
        for (; k < nc; ++k) {
            const uint32_t op = cg[k] & 0xF, l = cg[k] >> 4;
            if (op == 0 || op == 2 || op == 7 || op == 8) break;
            if (op == 3) n.x += (int32_t)l;
            else if (op == 1 || op == 4) n.y += (int32_t)l;
        }
        n.k = k < nc ? k : nc - 1;
    }
    for (;;) {
        const uint32_t op = cg[n.k] & 0xF, l = cg[n.k] >> 4;
        const bool cons_ref = op == 0 || op == 2 || op == 3 || op == 7 || op == 8;
        if (cons_ref && pos - n.x < (int32_t)l) break;
        if (n.k + 1 >= nc) break;
        if (op == 0 || op == 7 || op == 8 || op == 1 || op == 4) n.y += (int32_t)l;
        if (cons_ref) n.x += (int32_t)l;
        ++n.k;
    }
    const uint32_t op = cg[n.k] & 0xF;
    if (op == 2) return 1;
    if (op == 3) return 2;
    *qpos = n.y + (pos - n.x);
    return 0;
}

// growable 16-byte aligned key buffer (malloc'ed: pbf_keys_free releases it)
struct KeyBuf {
    uint16_t *p = nullptr;
    size_t n = 0, cap = 0;
    ~KeyBuf() { free(p); }
    bool reserve(size_t want) {
        if (want <= cap) return true;
        size_t nc = std::max<size_t>(want, cap + cap / 2 + 1024);
        nc = (nc + 7) & ~(size_t)7;
        uint16_t *q = (uint16_t *)aligned_alloc(16, nc * 2);
        if (!q) return false;
        if (n) memcpy(q, p, n * 2);
        free(p);
        p = q;
        cap = nc;
        return true;
    }
    uint16_t *release() {
        uint16_t *q = p;
        p = nullptr;
        n = cap = 0;
        return q;
    }
};

// Positions [cb, ce) of one walk of `rs` (every read kept: no maxcnt drop can occur) into a key
// batch: per position the reads that span it in file order (the pileup buffer), each resolved
// to a query position; deletions / ref skips / reads without RG are skipped, an RG without a
// sample is the reference's fatal error, the first max_depth reads of a sample are its reads,
// and call_base's per-read loop keeps those passing the baseQ / mapQ / N filters as keys.
// A read's per-position outcome is resolved once, when it joins the buffer: one u16 code per
// position it spans in [cb, ce) (0xFFFF: no base there -- deletion / ref skip; else its key, 0
// when call_base's filters drop it but it still counts against max_depth), so a position costs
// one code load per buffered read.
constexpr uint16_t kNoBase = 0xFFFF;
struct Act {
    const uint16_t *code;   // code[pos] for pos in [joined, end)
    int32_t end;
    int32_t sample;
    uint32_t mq2;
    uint32_t rec;           // index in rs.r
};
// call_base's key of a base as a function of (quality byte, nt16) for one (mapQ, strand): a
// 4096-entry table per pair, built when first needed
struct KeyLut {
    std::vector<std::vector<uint16_t>> t = std::vector<std::vector<uint16_t>>(512);
    const uint16_t *get(uint32_t mapq, uint32_t strand, uint32_t minb, uint32_t minm, bool ill) {
        std::vector<uint16_t> &v = t[(mapq << 1) | strand];
        if (v.empty()) {
            v.resize(4096);
            for (uint32_t q = 0; q < 256; ++q)
                for (uint32_t nt = 0; nt < 16; ++nt)
                    v[q << 4 | nt] = (uint16_t)pbg::read_to_key(q | mapq << 8 | nt << 16 | strand << 20, minb, minm, ill);
        }
        return v.data();
    }
};
int fast_walk(const RecSet &rs, int32_t cb, int32_t ce, const WalkCfg &cf, const pbf_filter &f, std::vector<uint16_t> &codes,
              KeyLut &lut, pbf_keys *out) {
    const int ns = cf.ns, kb = f.k_bytes;
    const uint32_t L = (uint32_t)(ce - cb);
    const uint32_t minb = (uint32_t)(f.min_baseQ & 0xff), minm = (uint32_t)(f.min_mapQ & 0xff);
    const bool ill = f.illumina != 0;
    const uint32_t md = (uint32_t)std::max(0, cf.max_depth);
    KeyBuf keys;
    // the codes of every read over [cb, ce): their total is the keys' upper bound
    size_t ncode = 0;
    for (const Rec2 &r : rs.r)
        if (!(r.tid < 0 || (r.flag & kDefMask)) && r.end > cb && r.pos < ce)
            ncode += (size_t)(std::min(r.end, ce) - std::max(r.pos, cb));
    if (codes.size() < ncode + 1) codes.resize(ncode + 1);
    if (!keys.reserve(ncode + 8)) return fail(PBF_E_IO, "out of host memory");
    size_t cfill = 0;
    const uint8_t *ar = rs.arena.data();
    // resolve_cigar2 + call_base's key for each position of [a, b) a read spans
    auto fill = [&](const Rec2 &r, int32_t a, int32_t b, uint16_t *dst) {
        const uint8_t *rec = ar + r.off;
        const uint32_t *cg = reinterpret_cast<const uint32_t *>(rec);
        const uint8_t *seq = rec + 4 * (size_t)r.n_cigar, *qual = seq + (r.l_seq + 1) / 2;
        const uint16_t *kl = lut.get(r.mapq, r.strand, minb, minm, ill);
        auto key_at = [&](int32_t qp) -> uint16_t {
            if (qp < 0 || qp >= r.l_seq) return 0;   // a CIGAR past its sequence (the reference reads past it)
            return kl[(uint32_t)qual[qp] << 4 | ((seq[qp >> 1] >> ((~qp & 1) << 2)) & 0xFu)];
        };
        const uint32_t op0 = cg[0] & 0xF;
        if (r.n_cigar == 1 && (op0 == 0 || op0 == 7 || op0 == 8)) {   // one M / = / X: query pos = p - pos
            const int32_t q1 = std::min(b - r.pos, r.l_seq);
            uint16_t *d = dst;
            int32_t qp = a - r.pos;
            if (qp < q1 && (qp & 1)) *d++ = key_at(qp++);
            for (; qp + 1 < q1; qp += 2) {   // two bases per sequence byte
                const uint32_t sb = seq[qp >> 1];
                d[0] = kl[(uint32_t)qual[qp] << 4 | (sb >> 4)];
                d[1] = kl[(uint32_t)qual[qp + 1] << 4 | (sb & 0xFu)];
                d += 2;
            }
            if (qp < q1) *d++ = key_at(qp++);
            for (int32_t p = r.pos + std::max(qp, q1); p < b; ++p) *d++ = 0;   // past the sequence
            return;
        }
        Cur cur{&r, -1, 0, 0};
        for (int32_t p = a; p < b; ++p) {
            int32_t qp = 0;
            const int kind = r.n_cigar ? resolve2(cur, cg, p, &qp) : 1;
            dst[p - a] = kind != 0 ? kNoBase : key_at(qp);
        }
    };
    // the buffer, split by sample (each list in file order = the buffer's order); reads without
    // RG never reach a sample but still make their positions called back (`cover`, a difference
    // array over [cb, ce]); a read whose RG has no sample is the fatal error at its first base
    std::vector<std::vector<Act>> lists(ns);
    for (auto &l : lists) l.reserve(64);
    // per list: the earliest end among its reads (no read leaves before it)
    std::vector<int32_t> minend((size_t)ns, INT32_MAX);
    std::vector<int32_t> cover((size_t)L + 1, 0);
    int64_t bad_pos = INT64_MAX;
    size_t bad_rec = 0;
    size_t idx = 0;
    const size_t nrec = rs.r.size();
    uint8_t *kout = (uint8_t *)out->k;
    uint32_t *rout = out->rmsq;
    int32_t live = 0;   // coverage at pos
    for (int32_t pos = cb; pos < ce;) {
        const uint32_t i = (uint32_t)(pos - cb);
        if ((i & 63u) == 0) out->block_off[i >> 6] = keys.n;
        // reads starting at or before pos join the buffer in file order
        while (idx < nrec && rs.r[idx].pos <= pos) {
            const Rec2 &r = rs.r[idx++];
            if (r.tid < 0 || (r.flag & kDefMask) || r.end <= pos) continue;
            const int32_t b = std::min(r.end, ce);
            ++cover[i];
            --cover[(uint32_t)(b - cb)];
            if (r.sample == -1) continue;   // no RG: skipped by the partition
            uint16_t *dst = codes.data() + cfill;
            fill(r, pos, b, dst);
            cfill += (size_t)(b - pos);
            if (r.sample < 0) {   // its first base in [pos, b), if any, is where the reference stops
                for (int32_t p = pos; p < b; ++p)
                    if (dst[p - pos] != kNoBase) {
                        if (p < bad_pos) bad_pos = p, bad_rec = idx - 1;
                        break;
                    }
                continue;
            }
            lists[r.sample].push_back(Act{dst - pos, b, r.sample, (uint32_t)r.mapq * r.mapq, (uint32_t)(idx - 1)});
            minend[r.sample] = std::min(minend[r.sample], b);
        }
        live += cover[i];
        if (live == 0) {   // no read spans pos: no callback until the next read starts
            const int32_t nxt = idx < nrec ? std::max(pos + 1, std::min(ce, rs.r[idx].pos)) : ce;
            for (int32_t q = pos + 1; q < nxt; ++q) {
                const uint32_t iq = (uint32_t)(q - cb);
                live += cover[iq];   // (zero: nothing starts or ends in between)
                if ((iq & 63u) == 0) out->block_off[iq >> 6] = keys.n;
            }
            pos = nxt;
            continue;
        }
        out->ref[i] &= 0x7F;   // a read spans pos: the pileup calls back here
        const size_t t0 = (size_t)i * ns;
        // compact pieces: the reference base index of an upper-case A/C/G/T position, else -1
        const int cmp_base = f.compact ? ref_base_upper(out->ref[i]) : -1;
        uint16_t *kd = keys.p + keys.n;
        size_t nk = 0;
        for (int s = 0; s < ns; ++s) {
            std::vector<Act> &l = lists[s];
            if (minend[s] <= pos) {   // some read finished: it leaves the buffer
                l.erase(std::remove_if(l.begin(), l.end(), [pos](const Act &a) { return a.end <= pos; }), l.end());
                int32_t me = INT32_MAX;
                for (const Act &a : l) me = std::min(me, a.end);
                minend[s] = me;
            }
            const size_t na = l.size();
            const Act *A = l.data();
            uint32_t kk = 0, rq = 0;
            if (na <= md) {   // max_depth cannot bind: every read with a base here is kept
                for (size_t j = 0; j < na; ++j) {
                    const uint16_t c = A[j].code[pos];
                    const bool key = c != 0 && c != kNoBase;   // a key (0: filtered; no base here)
                    kd[nk] = c;
                    nk += key;
                    kk += key;
                    rq += key ? A[j].mq2 : 0u;   // rmsq += SQ(core.qual) (popbam.cpp:287)
                }
            } else {
                uint32_t raw = 0;
                for (size_t j = 0; j < na; ++j) {
                    const uint16_t c = A[j].code[pos];
                    if (c == kNoBase || raw >= md) continue;   // no base here; past the sample's max_depth reads
                    ++raw;
                    kd[nk] = c;
                    nk += c != 0;
                    kk += c != 0;
                    rq += c ? A[j].mq2 : 0u;
                }
            }
            if (kb == 1) {
                if (kk > 255) return fail(PBF_E_ARG, "more than 255 keys per sample need k_bytes = 2");
                kout[t0 + s] = (uint8_t)kk;
            } else {
                reinterpret_cast<uint16_t *>(kout)[t0 + s] = (uint16_t)kk;
            }
            if (cmp_base >= 0 && kk >= 1 && kk <= 32 && all_on_base(kd + nk - kk, kk, (uint32_t)cmp_base)) {
                rq |= 0x80000000u;   // compact: reference-only, its keys left out
                nk -= kk;
            }
            rout[t0 + s] = rq;
        }
        keys.n += nk;
        ++pos;
    }
    out->block_off[(L + 63) / 64] = keys.n;
    out->n_keys = keys.n;
    out->keys = keys.release();
    if (bad_pos != INT64_MAX) {
        const Rec2 &r = rs.r[bad_rec];
        const char *rg = (const char *)ar + r.off + 4 * (size_t)r.n_cigar + (r.l_seq + 1) / 2 + r.l_seq;
        return fail(PBF_E_RG, std::string("Problem assigning read group ") + rg +
                                  " to a sample.\nPlease check BAM header for correct SM and PO tags");
    }
    return PBF_OK;
}

struct PieceProf {
    double t_fetch = 0, t_inflate = 0, t_walk = 0;
    uint64_t bytes_in = 0, bytes_out = 0, records = 0;
    uint32_t crowded = 0;
};

// one piece [cb, ce) of a region as a key batch: the fast walk, or (a read can meet a full
// buffer) the reference's window-by-window walks + pbf_pack
int piece_keys(pbf_bam *b, int tid, int32_t cb, int32_t ce, int32_t rbeg, int32_t rend, int32_t win,
               const char *refseq, const WalkCfg &cf, const pbf_filter &f, RecSet &rs, std::vector<uint16_t> &codes,
               KeyLut &lut, pbf_keys *out, PieceProf &pp) {
    memset(out, 0, sizeof(*out));
    const uint32_t L = (uint32_t)(ce - cb);
    const double inf0 = b->z.t_inflate;
    const uint64_t bi0 = b->z.bytes_in, bo0 = b->z.bytes_out;
    const auto t0 = Clock::now();
    const RgIndex rgi(cf);
    int r = fetch2(b, tid, std::max(0, cb - 1), ce, rgi, rs);
    if (r != PBF_OK) return r;
    int32_t lo = cb;
    for (const Rec2 &x : rs.r)
        if (!(x.flag & kDefMask)) lo = std::min(lo, x.pos);
    // the buffer bound of chunk_walk (max_buffer_bound) on the reads that reach cb
    int bound = 0;
    {
        std::vector<int32_t> ends;
        auto scan = [&](const Rec2 &x) {
            if (x.tid < 0 || (x.flag & kDefMask)) return;
            while (!ends.empty() && ends.front() < x.pos) {
                std::pop_heap(ends.begin(), ends.end(), std::greater<int32_t>());
                ends.pop_back();
            }
            if (x.pos >= cb || x.end >= cb) bound = std::max(bound, (int)ends.size());
            ends.push_back(std::max(x.end, x.pos + 1));
            std::push_heap(ends.begin(), ends.end(), std::greater<int32_t>());
        };
        if (lo < cb) {   // the reads before cb that reach it: their tests see reads ending before cb too
            RecSet early;
            r = fetch2(b, tid, std::max(0, lo - 1), cb, rgi, early);
            if (r != PBF_OK) return r;
            for (const Rec2 &x : early.r)
                if (x.pos < cb) scan(x);
        }
        for (const Rec2 &x : rs.r)
            if (lo >= cb || x.pos >= cb) scan(x);
    }
    const auto t1 = Clock::now();
    pp.t_fetch += secs(t0, t1);
    pp.records += rs.r.size();
    if (bound + 2 > kMaxCnt) {   // crowded: the reference's own walks, then call_base's per-read loop
        ++pp.crowded;
        pbf_batch raw;
        r = piece_batch(b, tid, cb, ce, rbeg, rend, win, refseq, cf, &raw);
        if (r == PBF_OK) {
            r = pbf_pack(&raw, cf.ns, &f, out);
            pbf_batch_free(&raw);
        }
    } else {
        const size_t nt = (size_t)L * cf.ns;
        out->n_sites = L;
        out->pos0 = cb;
        out->ref = (uint8_t *)malloc(std::max<size_t>(L, 1));
        out->k = calloc(std::max<size_t>(nt, 1), f.k_bytes);
        out->rmsq = (uint32_t *)calloc(std::max<size_t>(nt, 1), sizeof(uint32_t));
        out->block_off = (uint64_t *)calloc(L / 64 + 2, sizeof(uint64_t));
        if (!out->ref || !out->k || !out->rmsq || !out->block_off) {
            pbf_keys_free(out);
            return fail(PBF_E_IO, "out of host memory");
        }
        for (uint32_t i = 0; i < L; ++i) out->ref[i] = (uint8_t)refseq[cb + i] | 0x80;
        r = fast_walk(rs, cb, ce, cf, f, codes, lut, out);
        if (r != PBF_OK) pbf_keys_free(out);
    }
    pp.t_walk += secs(t1, Clock::now());
    pp.t_inflate += b->z.t_inflate - inf0;
    pp.bytes_in += b->z.bytes_in - bi0;
    pp.bytes_out += b->z.bytes_out - bo0;
    return r;
}

}  // namespace

// ---------------------------------------------------------------- piece stream
// Pieces of a region walked by worker threads (each with its own file handle) and handed out in
// position order; at most `lookahead` pieces wait, so host memory is bounded by the lookahead.
struct pbf_kstream {
    std::string path;
    int tid = 0;
    int32_t beg = 0, end = 0, win = 0, chunk = 0;
    int64_t nchunk = 0;
    const char *refseq = nullptr;
    WalkCfg cf;
    pbf_filter f{};
    std::vector<pbf_keys> parts;
    std::vector<int> state;        // 0 pending, 1 ready, 2 taken
    std::vector<int> rc;
    std::vector<std::string> msg;
    std::mutex m;
    std::condition_variable cv_ready, cv_space;
    int64_t next = 0, consumed = 0, lookahead = 0;
    bool stop = false;
    std::vector<std::thread> th;
    pbf_profile prof{};
    Clock::time_point t_open;
};

namespace {

void kstream_worker(pbf_kstream *ks) {
    pbf_bam *b = nullptr;
    int open_rc = pbf_open(&b, ks->path.c_str());
    if (open_rc == PBF_OK && ks->tid >= (int)b->names.size()) open_rc = fail(PBF_E_ARG, "bad argument");
    const std::string open_msg = open_rc ? g_err : std::string();
    RecSet rs;
    std::vector<uint16_t> codes;
    KeyLut lut;
    PieceProf pp;
    for (;;) {
        int64_t c;
        {
            std::unique_lock<std::mutex> lk(ks->m);
            ks->cv_space.wait(lk, [&] { return ks->stop || ks->next >= ks->nchunk || ks->next < ks->consumed + ks->lookahead; });
            if (ks->stop || ks->next >= ks->nchunk) break;
            c = ks->next++;
        }
        const int32_t cb = (int32_t)(ks->beg + c * (int64_t)ks->chunk);
        const int32_t ce = (int32_t)std::min<int64_t>(ks->end, ks->beg + (c + 1) * (int64_t)ks->chunk);
        pbf_keys out;
        memset(&out, 0, sizeof(out));
        int r = open_rc;
        std::string msg = open_msg;
        pp = PieceProf{};
        if (r == PBF_OK) {
            r = piece_keys(b, ks->tid, cb, ce, ks->beg, ks->end, ks->win, ks->refseq, ks->cf, ks->f, rs, codes, lut, &out, pp);
            if (r != PBF_OK) msg = g_err;
        }
        {
            std::lock_guard<std::mutex> lk(ks->m);
            ks->parts[c] = out;
            ks->rc[c] = r;
            ks->msg[c] = msg;
            ks->state[c] = 1;
            ks->prof.t_fetch += pp.t_fetch;
            ks->prof.t_inflate += pp.t_inflate;
            ks->prof.t_walk += pp.t_walk;
            ks->prof.bytes_compressed += pp.bytes_in;
            ks->prof.bytes_inflated += pp.bytes_out;
            ks->prof.records += pp.records;
            ks->prof.crowded_pieces += pp.crowded;
        }
        ks->cv_ready.notify_all();
    }
    if (b) pbf_close(b);
}

}  // namespace

extern "C" {

int pbf_kstream_open(const char *path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end, int32_t win_size,
                     const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg, int32_t fallback,
                     int ns, int max_depth, const pbf_filter *f, pbf_kstream **out) {
    if (!out) return fail(PBF_E_ARG, "bad argument");
    *out = nullptr;
    if (!path || !refseq || !f || ns < 1 || end < beg || n_threads < 1 || tid < 0 || (f->k_bytes != 1 && f->k_bytes != 2))
        return fail(PBF_E_ARG, "bad argument");
    pbf_kstream *ks = new pbf_kstream();
    ks->t_open = Clock::now();
    ks->path = path;
    ks->tid = tid;
    ks->beg = beg;
    ks->end = end;
    ks->win = win_size;
    if (chunk <= 0) chunk = 1 << 20;
    ks->chunk = (chunk + 63) / 64 * 64;   // piece borders on 64-position blocks: block_off concatenates
    ks->nchunk = std::max<int64_t>(1, ((int64_t)end - beg + ks->chunk - 1) / ks->chunk);
    if (end == beg) ks->nchunk = 1;
    ks->refseq = refseq;
    ks->cf = make_cfg(rg_ids, rg_sample, n_rg, fallback, ns, max_depth);
    ks->f = *f;
    ks->parts.assign((size_t)ks->nchunk, pbf_keys{});
    ks->state.assign((size_t)ks->nchunk, 0);
    ks->rc.assign((size_t)ks->nchunk, PBF_OK);
    ks->msg.assign((size_t)ks->nchunk, std::string());
    const int nt = (int)std::min<int64_t>(n_threads, ks->nchunk);
    ks->lookahead = std::max<int64_t>(2, 2 * (int64_t)nt);
    ks->prof.threads = nt;
    ks->prof.pieces = (uint32_t)ks->nchunk;
    for (int w = 0; w < nt; ++w) ks->th.emplace_back(kstream_worker, ks);
    *out = ks;
    return PBF_OK;
}

int pbf_kstream_next(pbf_kstream *ks, pbf_keys *piece) {
    if (!ks || !piece) return fail(PBF_E_ARG, "bad argument");
    memset(piece, 0, sizeof(*piece));
    std::unique_lock<std::mutex> lk(ks->m);
    if (ks->consumed >= ks->nchunk) return 0;
    const auto tw = Clock::now();
    // state 2 at `consumed` = a failed piece already reported: the error is sticky (every later
    // call returns it again instead of waiting for a piece that never comes)
    ks->cv_ready.wait(lk, [&] { return ks->state[ks->consumed] >= 1; });
    ks->prof.t_consumer_wait += secs(tw, Clock::now());
    const int64_t c = ks->consumed;
    ks->state[c] = 2;
    if (ks->rc[c] != PBF_OK) {   // the first failing piece in position order (the sequential walk's error)
        const int r = ks->rc[c];
        const std::string msg = ks->msg[c];
        lk.unlock();
        return fail(r, msg);
    }
    *piece = ks->parts[c];
    memset(&ks->parts[c], 0, sizeof(pbf_keys));
    ++ks->consumed;
    lk.unlock();
    ks->cv_space.notify_all();
    return 1;
}

int pbf_kstream_profile(pbf_kstream *ks, pbf_profile *p) {
    if (!ks || !p) return fail(PBF_E_ARG, "bad argument");
    std::lock_guard<std::mutex> lk(ks->m);
    *p = ks->prof;
    p->t_wall = secs(ks->t_open, Clock::now());
    return PBF_OK;
}

void pbf_kstream_close(pbf_kstream *ks) {
    if (!ks) return;
    {
        std::lock_guard<std::mutex> lk(ks->m);
        ks->stop = true;
    }
    ks->cv_space.notify_all();
    for (auto &t : ks->th) t.join();
    for (auto &p : ks->parts) pbf_keys_free(&p);
    delete ks;
}

}  // extern "C"

namespace {
}  // namespace

extern "C" {

int pbf_pileup(pbf_bam *b, int tid, int32_t beg, int32_t end, const char *refseq, const char *const *rg_ids,
               const int32_t *rg_sample, int n_rg, int32_t fallback, int ns, int max_depth, pbf_batch *out) {
    if (!b || !out || !refseq || ns < 1 || end < beg || tid < 0 || tid >= (int)b->names.size())
        return fail(PBF_E_ARG, "bad argument");
    const WalkCfg cf = make_cfg(rg_ids, rg_sample, n_rg, fallback, ns, max_depth);
    int r = batch_alloc(out, beg, (uint32_t)(end - beg), ns, refseq);
    if (r != PBF_OK) return r;
    std::vector<Rec> recs;
    WalkOut o{beg, (uint32_t)(end - beg), out->ref, out->depth, {}};
    r = fetch_region(b, tid, beg, end, recs);   // one bam_fetch + pileup of the region
    if (r == PBF_OK) r = walk(recs, beg, end, cf, o);
    if (r != PBF_OK) {
        pbf_batch_free(out);
        return r;
    }
    return batch_finish(out, ns, o.reads);
}

int pbf_pileup_mt(const char *path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end, int32_t win_size,
                  const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg,
                  int32_t fallback, int ns, int max_depth, pbf_batch *out) {
    if (!path || !out || !refseq || ns < 1 || end < beg || n_threads < 1 || tid < 0)
        return fail(PBF_E_ARG, "bad argument");
    memset(out, 0, sizeof(*out));
    const WalkCfg cf = make_cfg(rg_ids, rg_sample, n_rg, fallback, ns, max_depth);
    const int64_t L = (int64_t)end - beg;
    if (chunk <= 0) chunk = 1 << 20;
    chunk = (chunk + 63) / 64 * 64;   // chunk borders on 64-position blocks: block_off concatenates
    const int64_t nchunk = std::max<int64_t>(1, (L + chunk - 1) / chunk);
    std::vector<pbf_batch> parts((size_t)nchunk);
    std::vector<int> rc((size_t)nchunk, PBF_OK);
    std::vector<std::string> msg((size_t)nchunk);
    for (auto &p : parts) memset(&p, 0, sizeof(p));
    const int nt = (int)std::min<int64_t>(n_threads, nchunk);
    auto worker = [&](int w) {
        pbf_bam *b = nullptr;
        int r = pbf_open(&b, path);
        if (r == PBF_OK && tid >= (int)b->names.size()) r = fail(PBF_E_ARG, "bad argument");
        for (int64_t c = w; c < nchunk; c += nt) {
            if (r == PBF_OK) {
                const int32_t cb = (int32_t)(beg + c * chunk), ce = (int32_t)std::min<int64_t>(end, beg + (c + 1) * chunk);
                r = piece_batch(b, tid, cb, ce, beg, end, win_size, refseq, cf, &parts[c]);
            }
            rc[c] = r;
            if (r != PBF_OK) msg[c] = g_err;
        }
        if (b) pbf_close(b);
    };
    std::vector<std::thread> th;
    for (int w = 1; w < nt; ++w) th.emplace_back(worker, w);
    worker(0);
    for (auto &t : th) t.join();
    // first failing chunk in position order = the error a sequential walk meets first
    for (int64_t c = 0; c < nchunk; ++c)
        if (rc[c] != PBF_OK) {
            for (auto &p : parts) pbf_batch_free(&p);
            return fail(rc[c], msg[c]);
        }
    uint64_t n_reads = 0;
    for (auto &p : parts) n_reads += p.n_reads;
    out->n_sites = (uint32_t)L;
    out->pos0 = beg;
    out->n_reads = n_reads;
    out->ref = (uint8_t *)malloc(std::max<size_t>((size_t)L, 1));
    out->depth = (uint16_t *)malloc(std::max<size_t>((size_t)L * ns, 1) * sizeof(uint16_t));
    out->block_off = (uint64_t *)calloc((size_t)L / 64 + 2, sizeof(uint64_t));
    out->reads = (uint32_t *)malloc(std::max<uint64_t>(n_reads, 1) * sizeof(uint32_t));
    if (!out->ref || !out->depth || !out->block_off || !out->reads) {
        for (auto &p : parts) pbf_batch_free(&p);
        pbf_batch_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    size_t site = 0;
    uint64_t roff = 0;
    for (auto &p : parts) {
        if (p.n_sites) {
            memcpy(out->ref + site, p.ref, p.n_sites);
            memcpy(out->depth + site * ns, p.depth, (size_t)p.n_sites * ns * sizeof(uint16_t));
            for (uint32_t bk = 0; bk * 64 < p.n_sites; ++bk) out->block_off[site / 64 + bk] = roff + p.block_off[bk];
        }
        if (p.n_reads) memcpy(out->reads + roff, p.reads, p.n_reads * sizeof(uint32_t));
        site += p.n_sites;
        roff += p.n_reads;
        pbf_batch_free(&p);
    }
    out->block_off[((size_t)L + 63) / 64] = roff;
    return PBF_OK;
}

void pbf_keys_free(pbf_keys *o) {
    if (!o) return;
    free(o->ref);
    free(o->k);
    free(o->rmsq);
    free(o->block_off);
    free(o->keys);
    memset(o, 0, sizeof(*o));
}

int pbf_pack(const pbf_batch *raw, int ns, const pbf_filter *f, pbf_keys *out) {
    if (!raw || !f || !out || ns < 1 || (f->k_bytes != 1 && f->k_bytes != 2)) return fail(PBF_E_ARG, "bad argument");
    memset(out, 0, sizeof(*out));
    const uint32_t L = raw->n_sites;
    const size_t nt = (size_t)L * ns;
    const int kb = f->k_bytes;
    out->n_sites = L;
    out->pos0 = raw->pos0;
    out->ref = (uint8_t *)malloc(std::max<size_t>(L, 1));
    out->k = calloc(std::max<size_t>(nt, 1), kb);
    out->rmsq = (uint32_t *)calloc(std::max<size_t>(nt, 1), sizeof(uint32_t));
    out->block_off = (uint64_t *)calloc(L / 64 + 2, sizeof(uint64_t));
    out->keys = (uint16_t *)aligned_alloc(16, (std::max<uint64_t>(raw->n_reads, 1) * 2 + 15) & ~(size_t)15);
    if (!out->ref || !out->k || !out->rmsq || !out->block_off || !out->keys) {
        pbf_keys_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    if (L) memcpy(out->ref, raw->ref, L);
    const uint32_t minb = (uint32_t)(f->min_baseQ & 0xff), minm = (uint32_t)(f->min_mapQ & 0xff);
    const bool ill = f->illumina != 0;
    uint64_t r = 0, nk = 0;
    for (size_t t = 0; t < nt; ++t) {
        if (t % ((size_t)64 * ns) == 0) out->block_off[t / ((size_t)64 * ns)] = nk;
        const uint32_t d = raw->depth[t];
        uint32_t kk = 0, rq = 0;
        for (uint32_t j = 0; j < d; ++j, ++r) {
            const uint32_t w = raw->reads[r];
            const uint32_t key = pbg::read_to_key(w, minb, minm, ill);
            if (!key) continue;
            out->keys[nk++] = (uint16_t)key;
            const uint32_t mq = (w >> 8) & 0xffu;
            rq += mq * mq;   // rmsq += SQ(core.qual) (popbam.cpp:287)
            ++kk;
        }
        if (kb == 1) {
            if (kk > 255) {
                pbf_keys_free(out);
                return fail(PBF_E_ARG, "more than 255 keys per sample need k_bytes = 2");
            }
            ((uint8_t *)out->k)[t] = (uint8_t)kk;
        } else {
            ((uint16_t *)out->k)[t] = (uint16_t)kk;
        }
        const uint8_t rc = raw->ref[t / ns];
        const int cb = f->compact && !(rc & 0x80) ? ref_base_upper(rc) : -1;
        if (cb >= 0 && kk >= 1 && kk <= 32 && all_on_base(out->keys + nk - kk, kk, (uint32_t)cb)) {
            rq |= 0x80000000u;   // compact: reference-only, its keys left out
            nk -= kk;
        }
        out->rmsq[t] = rq;
    }
    if (r != raw->n_reads) {
        pbf_keys_free(out);
        return fail(PBF_E_ARG, "depth[] does not add up to n_reads");
    }
    out->block_off[(L + 63) / 64] = nk;
    out->n_keys = nk;
    return PBF_OK;
}

int pbf_compact(const pbf_keys *in, int ns, int kb, pbf_keys *out) {
    if (!in || !out || ns < 1 || (kb != 1 && kb != 2)) return fail(PBF_E_ARG, "bad argument");
    memset(out, 0, sizeof(*out));
    const uint32_t L = in->n_sites;
    const size_t nt = (size_t)L * ns;
    const uint32_t nblk = (L + 63) / 64;
    out->n_sites = L;
    out->pos0 = in->pos0;
    out->ref = (uint8_t *)malloc(std::max<size_t>(L, 1));
    out->k = malloc(std::max<size_t>(nt, 1) * kb);
    out->rmsq = (uint32_t *)malloc(std::max<size_t>(nt, 1) * sizeof(uint32_t));
    out->block_off = (uint64_t *)calloc(nblk + 2, sizeof(uint64_t));
    const uint64_t k0 = in->block_off[0], ktot = in->block_off[nblk] - k0;
    out->keys = (uint16_t *)aligned_alloc(16, (std::max<uint64_t>(ktot, 1) * 2 + 15) & ~(size_t)15);
    if (!out->ref || !out->k || !out->rmsq || !out->block_off || !out->keys) {
        pbf_keys_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    if (L) memcpy(out->ref, in->ref, L);
    memcpy(out->k, in->k, nt * kb);
    const uint16_t *src = in->keys + k0;   // offsets may be absolute (include/popbam_gpu.h)
    uint64_t r = 0, nk = 0;
    for (size_t t = 0; t < nt; ++t) {
        if (t % ((size_t)64 * ns) == 0) out->block_off[t / ((size_t)64 * ns)] = nk;
        const uint32_t kk = kb == 1 ? ((const uint8_t *)in->k)[t] : ((const uint16_t *)in->k)[t];
        uint32_t rq = in->rmsq[t];
        const uint8_t rc = in->ref[t / ns];
        const int cb = !(rc & 0x80) ? ref_base_upper(rc) : -1;
        if (rq >> 31) {
            pbf_keys_free(out);
            return fail(PBF_E_ARG, "a sum of mapQ^2 reaches bit 31: no compact form");
        }
        if (cb >= 0 && kk >= 1 && kk <= 32 && all_on_base(src + r, kk, (uint32_t)cb)) {
            rq |= 0x80000000u;
        } else {
            memcpy(out->keys + nk, src + r, (size_t)kk * 2);
            nk += kk;
        }
        r += kk;
        out->rmsq[t] = rq;
    }
    if (r != ktot) {
        pbf_keys_free(out);
        return fail(PBF_E_ARG, "block_off does not add up to k[]");
    }
    out->block_off[nblk] = nk;
    out->n_keys = nk;
    return PBF_OK;
}

int pbf_pileup_keys_mt(const char *path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end,
                       int32_t win_size, const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg,
                       int32_t fallback, int ns, int max_depth, const pbf_filter *f, pbf_keys *out) {
    if (!path || !out || !refseq || !f || ns < 1 || end < beg || n_threads < 1 || tid < 0)
        return fail(PBF_E_ARG, "bad argument");
    memset(out, 0, sizeof(*out));
    pbf_kstream *ks = nullptr;
    int r = pbf_kstream_open(path, n_threads, chunk, tid, beg, end, win_size, refseq, rg_ids, rg_sample, n_rg, fallback, ns,
                             max_depth, f, &ks);
    if (r != PBF_OK) return r;
    std::vector<pbf_keys> parts;
    pbf_keys p;
    while ((r = pbf_kstream_next(ks, &p)) == 1) parts.push_back(p);
    const std::string msg = r < 0 ? g_err : std::string();
    pbf_kstream_close(ks);
    if (r < 0) {   // the first failing piece in position order
        for (auto &q : parts) pbf_keys_free(&q);
        return fail(r, msg);
    }
    const int64_t L = (int64_t)end - beg;
    uint64_t n_keys = 0;
    for (auto &q : parts) n_keys += q.n_keys;
    const int kb = f->k_bytes;
    out->n_sites = (uint32_t)L;
    out->pos0 = beg;
    out->n_keys = n_keys;
    out->ref = (uint8_t *)malloc(std::max<size_t>((size_t)L, 1));
    out->k = malloc(std::max<size_t>((size_t)L * ns, 1) * kb);
    out->rmsq = (uint32_t *)malloc(std::max<size_t>((size_t)L * ns, 1) * sizeof(uint32_t));
    out->block_off = (uint64_t *)calloc((size_t)L / 64 + 2, sizeof(uint64_t));
    out->keys = (uint16_t *)aligned_alloc(16, (std::max<uint64_t>(n_keys, 1) * 2 + 15) & ~(size_t)15);
    if (!out->ref || !out->k || !out->rmsq || !out->block_off || !out->keys) {
        for (auto &q : parts) pbf_keys_free(&q);
        pbf_keys_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    size_t site = 0;
    uint64_t koff = 0;
    for (auto &q : parts) {   // each part is released as soon as it is copied
        if (q.n_sites) {
            memcpy(out->ref + site, q.ref, q.n_sites);
            memcpy((char *)out->k + site * ns * kb, q.k, (size_t)q.n_sites * ns * kb);
            memcpy(out->rmsq + site * ns, q.rmsq, (size_t)q.n_sites * ns * sizeof(uint32_t));
            for (uint32_t bk = 0; bk * 64 < q.n_sites; ++bk) out->block_off[site / 64 + bk] = koff + q.block_off[bk];
        }
        if (q.n_keys) memcpy(out->keys + koff, q.keys, q.n_keys * sizeof(uint16_t));
        site += q.n_sites;
        koff += q.n_keys;
        pbf_keys_free(&q);
    }
    out->block_off[((size_t)L + 63) / 64] = koff;
    return PBF_OK;
}

int pbf_fasta_fetch(const char *fa_path, const char *name, char **seq, int64_t *len) {
    if (!fa_path || !name || !seq || !len) return fail(PBF_E_ARG, "null argument");
    *seq = nullptr;
    *len = 0;
    // .fai: name, length, offset, line bases, line width
    std::string fai = std::string(fa_path) + ".fai";
    FILE *fi = fopen(fai.c_str(), "r");
    FILE *f = fopen(fa_path, "rb");
    if (!f) {
        if (fi) fclose(fi);
        return fail(PBF_E_IO, std::string("cannot open ") + fa_path);
    }
    std::string out;
    bool found = false;
    if (fi) {
        char nm[4096];
        long long ln, off, lb, lw;
        while (fscanf(fi, "%4095s %lld %lld %lld %lld", nm, &ln, &off, &lb, &lw) == 5) {
            if (strcmp(nm, name) != 0) continue;
            found = true;
            out.reserve((size_t)ln);
            if (fseeko(f, (off_t)off, SEEK_SET) != 0) break;
            int c;
            while ((long long)out.size() < ln && (c = fgetc(f)) != EOF)
                if (c != '\n' && c != '\r') out.push_back((char)c);
            break;
        }
        fclose(fi);
    }
    if (!found) {   // scan: first header whose first word is `name`
        rewind(f);
        char *line = nullptr;
        size_t cap = 0;
        ssize_t n;
        bool in = false;
        while ((n = getline(&line, &cap, f)) > 0) {
            while (n > 0 && (line[n - 1] == '\n' || line[n - 1] == '\r')) line[--n] = 0;
            if (line[0] == '>') {
                if (in) break;
                std::string h(line + 1);
                h = h.substr(0, h.find_first_of(" \t"));
                in = h == name;
                found |= in;
                continue;
            }
            if (in) out.append(line, (size_t)n);
        }
        free(line);
    }
    fclose(f);
    if (!found) return fail(PBF_E_ARG, std::string("sequence ") + name + " not in " + fa_path);
    *seq = (char *)malloc(out.size() + 1);
    if (!*seq) return fail(PBF_E_IO, "out of host memory");
    memcpy(*seq, out.data(), out.size());
    (*seq)[out.size()] = 0;
    *len = (int64_t)out.size();
    return PBF_OK;
}

}  // extern "C"
