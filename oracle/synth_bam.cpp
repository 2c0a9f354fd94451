// synth_bam.cpp -- BAM + BAI + FASTA of the synthetic genome (TEST INFRASTRUCTURE, built into
// liboracle.so).  The same files tests/ref_baseline.make_inputs used to write record by record
// in Python (tests/golden/bamwriter.py): the genotypes behind the benchmark's pileup
// (orc_synth_genotypes), 100 bp `100M` reads every `step` bp per sample, one haplotype per read
// alternating, mapQ 60, baseQ 40, reverse strand on every other pair of reads, @RG per sample
// and two contiguous populations -- so POPBAM itself (the CPU baseline) and the drop-in command
// line read one BAM of any length.  Written from the SAM/BAM v1 specification: BGZF members of
// at most 0xFF00 bytes compressed in parallel (raw deflate level 1), the BAI binning index and
// 16 kbp linear index.  Nothing in the product writes BAM.
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <map>
#include <string>
#include <thread>
#include <vector>

extern "C" void orc_synth_genotypes(uint64_t seed, int32_t contig, uint64_t pos_lo, uint32_t L, int32_t n,
                                    uint8_t *ref, uint8_t *alleles);

namespace {

constexpr size_t kBlock = 0xFF00;

int reg2bin(int beg, int end) {   // SAM spec 5.3 (end exclusive)
    --end;
    if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
    if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
    if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
    if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
    if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
    return 0;
}

void put32(std::vector<uint8_t> &b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
void put16(std::vector<uint8_t> &b, uint16_t v) {
    b.push_back((uint8_t)v);
    b.push_back((uint8_t)(v >> 8));
}

// one BGZF member of `n` bytes (raw deflate, level 1)
std::vector<uint8_t> bgzf_member(const uint8_t *p, size_t n) {
    std::vector<uint8_t> out(18 + compressBound((uLong)n) + 8 + 64);
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    zs.next_in = const_cast<uint8_t *>(p);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data() + 18;
    zs.avail_out = (uInt)(out.size() - 18 - 8);
    deflate(&zs, Z_FINISH);
    const size_t cl = zs.total_out;
    deflateEnd(&zs);
    const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 0, 0};
    memcpy(out.data(), hdr, 18);
    const uint32_t bsize = (uint32_t)(cl + 25);   // BSIZE: the member's total size - 1
    out[16] = (uint8_t)(bsize & 0xFF);
    out[17] = (uint8_t)(bsize >> 8);
    const uint32_t crc = (uint32_t)crc32(0, p, (uInt)n);
    uint8_t *t = out.data() + 18 + cl;
    for (int i = 0; i < 4; ++i) t[i] = (uint8_t)(crc >> (8 * i));
    for (int i = 0; i < 4; ++i) t[4 + i] = (uint8_t)(n >> (8 * i));
    out.resize(18 + cl + 8);
    return out;
}

}  // namespace

extern "C" int orc_write_synth_bam(const char *dir, uint64_t seed, uint32_t L, int32_t n, int32_t npops, int32_t read_len,
                                   int32_t step, int32_t threads) {
    if (!dir || n < 1 || npops < 1 || read_len < 1 || step < 1 || L < (uint32_t)read_len) return -1;
    std::vector<uint8_t> ref(L), al((size_t)L * n);
    orc_synth_genotypes(seed, 0, 0, L, n, ref.data(), al.data());
    const std::string d(dir);
    {   // ref.fa, 60 bases per line
        FILE *f = fopen((d + "/ref.fa").c_str(), "wb");
        if (!f) return -2;
        fputs(">chr1\n", f);
        for (uint32_t i = 0; i < L; i += 60) {
            fwrite(ref.data() + i, 1, std::min<uint32_t>(60, L - i), f);
            fputc('\n', f);
        }
        fclose(f);
        // ref.fa.fai (faidx: name, length, offset, bases per line, bytes per line), written here
        // so that no reader builds it -- POPBAM's fai_load writes it on first use, which concurrent
        // region-sharded processes would race on
        FILE *fi = fopen((d + "/ref.fa.fai").c_str(), "wb");
        if (!fi) return -2;
        fprintf(fi, "chr1\t%u\t6\t60\t61\n", L);
        fclose(fi);
    }
    // header block (records start on a fresh member, as samtools writes)
    std::string text = "@HD\tVN:1.0\tSO:coordinate\n@SQ\tSN:chr1\tLN:" + std::to_string(L) + "\n";
    const int per = n / npops;
    for (int s = 0; s < n; ++s)
        text += "@RG\tID:rg" + std::to_string(s) + "\tSM:s" + std::to_string(s) + "\tPO:pop" +
                std::to_string(std::min(s / std::max(per, 1), npops - 1)) + "\n";
    std::vector<uint8_t> hdr = {'B', 'A', 'M', 1};
    put32(hdr, (uint32_t)text.size());
    hdr.insert(hdr.end(), text.begin(), text.end());
    put32(hdr, 1);
    put32(hdr, 5);
    const char nm[5] = {'c', 'h', 'r', '1', 0};
    hdr.insert(hdr.end(), nm, nm + 5);
    put32(hdr, L);
    // records in (pos, sample) order: the stable sort by pos of the per-sample read lists
    static const uint8_t kNt16[4] = {1, 2, 4, 8};
    std::vector<uint8_t> body;
    body.reserve((size_t)L / step * n * (36 + 16 + 4 + read_len / 2 + read_len + 8) + 64);
    struct Idx {
        uint64_t ubeg, uend;   // offsets in the uncompressed record stream
        int32_t pos, end;
    };
    std::vector<Idx> idx;
    idx.reserve((size_t)L / step * n + 16);
    for (uint32_t p = 0; p + (uint32_t)read_len <= L; ++p) {
        for (int s = 0; s < n; ++s) {
            if ((int)(p % (uint32_t)step) != s % step) continue;
            const uint32_t i = (p - (uint32_t)(s % step)) / (uint32_t)step;
            const int h = (int)((i + (uint32_t)s) & 1u);
            const std::string name = "r" + std::to_string(s) + "_" + std::to_string(i);
            const std::string rg = "rg" + std::to_string(s);
            const uint16_t flag = ((i >> 1) & 1u) ? 16 : 0;
            const size_t start = body.size();
            put32(body, 0);   // block_size, patched below
            put32(body, 0);   // tid
            put32(body, p);
            body.push_back((uint8_t)(name.size() + 1));
            body.push_back(60);   // mapq
            put16(body, (uint16_t)reg2bin((int)p, (int)p + read_len));
            put16(body, 1);       // n_cigar
            put16(body, flag);
            put32(body, (uint32_t)read_len);
            put32(body, 0xFFFFFFFFu);
            put32(body, 0xFFFFFFFFu);
            put32(body, 0);
            body.insert(body.end(), name.begin(), name.end());
            body.push_back(0);
            put32(body, (uint32_t)read_len << 4);   // 100M
            for (int j = 0; j < read_len; j += 2) {
                const uint8_t a = kNt16[(al[(size_t)(p + j) * n + s] >> (2 * h)) & 3];
                const uint8_t b = j + 1 < read_len ? kNt16[(al[(size_t)(p + j + 1) * n + s] >> (2 * h)) & 3] : 0;
                body.push_back((uint8_t)(a << 4 | b));
            }
            body.insert(body.end(), (size_t)read_len, (uint8_t)40);
            body.push_back('R');
            body.push_back('G');
            body.push_back('Z');
            body.insert(body.end(), rg.begin(), rg.end());
            body.push_back(0);
            const uint32_t bs = (uint32_t)(body.size() - start - 4);
            for (int k = 0; k < 4; ++k) body[start + k] = (uint8_t)(bs >> (8 * k));
            idx.push_back({start, body.size(), (int32_t)p, (int32_t)p + read_len});
        }
    }
    // members: the header alone, then the record stream in kBlock pieces, compressed in parallel
    const size_t nblk = (body.size() + kBlock - 1) / kBlock;
    std::vector<std::vector<uint8_t>> mem(nblk);
    {
        const int nt = std::max(1, std::min<int>(threads, 64));
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (size_t b = (size_t)t; b < nblk; b += (size_t)nt)
                    mem[b] = bgzf_member(body.data() + b * kBlock, std::min(kBlock, body.size() - b * kBlock));
            });
        for (auto &x : th) x.join();
    }
    const std::vector<uint8_t> hmem = bgzf_member(hdr.data(), hdr.size());
    std::vector<uint64_t> coff(nblk + 1);
    coff[0] = hmem.size();
    for (size_t b = 0; b < nblk; ++b) coff[b + 1] = coff[b] + mem[b].size();
    auto voff = [&](uint64_t u) {   // virtual offset of uncompressed record-stream byte u
        const size_t b = (size_t)(u / kBlock);
        return b < nblk ? (coff[b] << 16) | (u % kBlock) : (coff[nblk] << 16);
    };
    {
        FILE *f = fopen((d + "/in.bam").c_str(), "wb");
        if (!f) return -2;
        fwrite(hmem.data(), 1, hmem.size(), f);
        for (auto &m : mem) fwrite(m.data(), 1, m.size(), f);
        static const uint8_t kEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43, 2, 0,
                                         0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        fwrite(kEof, 1, 28, f);
        fclose(f);
    }
    // BAI: bins -> chunks (merged when adjacent), 16 kbp linear index
    std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
    std::map<int, uint64_t> lin;
    for (const Idx &x : idx) {
        const uint64_t bv = voff(x.ubeg), ev = voff(x.uend);
        auto &ch = bins[(uint32_t)reg2bin(x.pos, x.end)];
        if (!ch.empty() && ch.back().second == bv) ch.back().second = ev;
        else ch.emplace_back(bv, ev);
        for (int w = x.pos >> 14; w <= (x.end - 1) >> 14; ++w) {
            auto it = lin.find(w);
            if (it == lin.end() || bv < it->second) lin[w] = bv;
        }
    }
    std::vector<uint8_t> bai = {'B', 'A', 'I', 1};
    put32(bai, 1);
    put32(bai, (uint32_t)bins.size());
    for (auto &kv : bins) {
        put32(bai, kv.first);
        put32(bai, (uint32_t)kv.second.size());
        for (auto &c : kv.second) {
            put32(bai, (uint32_t)c.first);
            put32(bai, (uint32_t)(c.first >> 32));
            put32(bai, (uint32_t)c.second);
            put32(bai, (uint32_t)(c.second >> 32));
        }
    }
    const int n_intv = lin.empty() ? 0 : lin.rbegin()->first + 1;
    put32(bai, (uint32_t)n_intv);
    uint64_t prev = 0;
    for (int i = 0; i < n_intv; ++i) {
        auto it = lin.find(i);
        const uint64_t v = it != lin.end() ? it->second : prev;
        prev = v;
        put32(bai, (uint32_t)v);
        put32(bai, (uint32_t)(v >> 32));
    }
    FILE *f = fopen((d + "/in.bam.bai").c_str(), "wb");
    if (!f) return -2;
    fwrite(bai.data(), 1, bai.size(), f);
    fclose(f);
    return 0;
}
