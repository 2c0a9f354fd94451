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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <thread>
#include <string>
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

// ---------------------------------------------------------------- BGZF
struct Bgzf {
    FILE *f = nullptr;
    std::vector<uint8_t> blk;     // uncompressed current block
    size_t at = 0;                // read position in blk
    uint64_t blk_addr = 0;        // file offset of the current block
    uint64_t next_addr = 0;       // file offset of the next block
    std::vector<uint8_t> cbuf;

    ~Bgzf() {
        if (f) fclose(f);
    }
    // loads the block at file offset `addr`; false at EOF, throws nothing
    int load(uint64_t addr) {
        if (fseeko(f, (off_t)addr, SEEK_SET) != 0) return fail(PBF_E_IO, "seek failed");
        uint8_t h[18];
        size_t got = fread(h, 1, 18, f);
        blk.clear();
        at = 0;
        blk_addr = addr;
        if (got == 0) {
            next_addr = addr;
            return 0;   // EOF
        }
        if (got < 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4))
            return fail(PBF_E_FORMAT, "not a BGZF block");
        const int xlen = h[10] | h[11] << 8;
        std::vector<uint8_t> extra(xlen);
        memcpy(extra.data(), h + 12, std::min(xlen, 6));
        if (xlen > 6 && fread(extra.data() + 6, 1, xlen - 6, f) != (size_t)(xlen - 6))
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
        blk.resize(isize);
        next_addr = addr + (uint64_t)bsize + 1;
        if (isize == 0) return 1;
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        if (inflateInit2(&zs, -15) != Z_OK) return fail(PBF_E_FORMAT, "inflateInit2");
        zs.next_in = cbuf.data();
        zs.avail_in = (uInt)cdata;
        zs.next_out = blk.data();
        zs.avail_out = isize;
        const int r = inflate(&zs, Z_FINISH);
        inflateEnd(&zs);
        if (r != Z_STREAM_END || zs.avail_out != 0) return fail(PBF_E_FORMAT, "corrupt BGZF block");
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
            if (at >= blk.size()) {
                const int r = load(next_addr);
                if (r < 0) return r;
                if (r == 0) break;
                continue;
            }
            const size_t k = std::min(n - done, blk.size() - at);
            memcpy(o + done, blk.data() + at, k);
            at += k;
            done += k;
        }
        return (long)done;
    }
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

int pbf_pileup_keys_mt(const char *path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end,
                       int32_t win_size, const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg,
                       int32_t fallback, int ns, int max_depth, const pbf_filter *f, pbf_keys *out) {
    if (!path || !out || !refseq || !f || ns < 1 || end < beg || n_threads < 1 || tid < 0)
        return fail(PBF_E_ARG, "bad argument");
    memset(out, 0, sizeof(*out));
    const WalkCfg cf = make_cfg(rg_ids, rg_sample, n_rg, fallback, ns, max_depth);
    const int64_t L = (int64_t)end - beg;
    if (chunk <= 0) chunk = 1 << 20;
    chunk = (chunk + 63) / 64 * 64;   // chunk borders on 64-position blocks: block_off concatenates
    const int64_t nchunk = std::max<int64_t>(1, (L + chunk - 1) / chunk);
    std::vector<pbf_keys> parts((size_t)nchunk);
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
                pbf_batch raw;
                r = piece_batch(b, tid, cb, ce, beg, end, win_size, refseq, cf, &raw);
                if (r == PBF_OK) {
                    r = pbf_pack(&raw, ns, f, &parts[c]);
                    pbf_batch_free(&raw);
                }
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
    for (int64_t c = 0; c < nchunk; ++c)
        if (rc[c] != PBF_OK) {
            for (auto &p : parts) pbf_keys_free(&p);
            return fail(rc[c], msg[c]);
        }
    uint64_t n_keys = 0;
    for (auto &p : parts) n_keys += p.n_keys;
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
        for (auto &p : parts) pbf_keys_free(&p);
        pbf_keys_free(out);
        return fail(PBF_E_IO, "out of host memory");
    }
    size_t site = 0;
    uint64_t koff = 0;
    for (auto &p : parts) {   // each part is released as soon as it is copied
        if (p.n_sites) {
            memcpy(out->ref + site, p.ref, p.n_sites);
            memcpy((char *)out->k + site * ns * kb, p.k, (size_t)p.n_sites * ns * kb);
            memcpy(out->rmsq + site * ns, p.rmsq, (size_t)p.n_sites * ns * sizeof(uint32_t));
            for (uint32_t bk = 0; bk * 64 < p.n_sites; ++bk) out->block_off[site / 64 + bk] = koff + p.block_off[bk];
        }
        if (p.n_keys) memcpy(out->keys + koff, p.keys, p.n_keys * sizeof(uint16_t));
        site += p.n_sites;
        koff += p.n_keys;
        pbf_keys_free(&p);
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
