// call_kernel.hip -- per-position consensus call on gfx950 (the "pop_snp" stage).
//
// One workgroup (256 threads = 4 wave64) per PBG_SITE_BLOCK (64) positions.  The block's
// reads are one contiguous slice of the pileup batch; it is staged into LDS with 16-byte
// coalesced loads, then each thread takes (position, sample) tasks and runs
//   call_base per sample   popbam.cpp:252-306   (filters, keys, rms)
//   errmod_cal             pop_utils.cpp:280-365 (sorted keys, double accumulation)
//   gl2cns                 pop_utils.cpp:66-100
//   clean_heterozygotes    pop_utils.cpp:170-201  (per sample)
//   segbase / qfilter      pop_utils.cpp:122-168, 102-120 (per-sample parts)
// and one thread per position folds the samples into the packed row
// (fq, counted, cal_site_type: popbam.cpp:173-184, pop_nucdiv.cpp:168-196).
//
// Numerics follow the reference bit for bit: double accumulation of fk*beta in descending
// key order, float narrowing at every `float += double`, float sqrt for rms; the library is
// compiled with -ffp-contract=off so no FMA is formed (x86 SSE2 reference has none).
#include "pbg_common.h"

namespace pbg {

namespace {

__constant__ int kNt16Nt4[16] = {4, 0, 1, 4, 2, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4};

__device__ __forceinline__ unsigned char iupac_rev(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 14;
    }
}
// iupac[] (popbam.cpp:11) for the homozygous genotypes segbase compares with the reference
__device__ __forceinline__ char iupac_hom(unsigned g) {
    return g == 0 ? 'A' : g == 5 ? 'C' : g == 10 ? 'G' : 'T';
}

__device__ __forceinline__ void cswap(uint32_t &a, uint32_t &b) {  // descending
    uint32_t hi = a > b ? a : b, lo = a > b ? b : a;
    a = hi;
    b = lo;
}

// 16-input Batcher odd-even merge sorting network (63 comparators), descending.  Verified
// exhaustively by the 0-1 principle in tests/test_kernel_source.py.
__device__ __forceinline__ void sort16_desc(uint32_t *k) {
#define CS(i, j) cswap(k[i], k[j])
    CS(0, 1); CS(2, 3); CS(0, 2); CS(1, 3); CS(1, 2); CS(4, 5); CS(6, 7); CS(4, 6);
    CS(5, 7); CS(5, 6); CS(0, 4); CS(2, 6); CS(2, 4); CS(1, 5); CS(3, 7); CS(3, 5);
    CS(1, 2); CS(3, 4); CS(5, 6); CS(8, 9); CS(10, 11); CS(8, 10); CS(9, 11); CS(9, 10);
    CS(12, 13); CS(14, 15); CS(12, 14); CS(13, 15); CS(13, 14); CS(8, 12); CS(10, 14); CS(10, 12);
    CS(9, 13); CS(11, 15); CS(11, 13); CS(9, 10); CS(11, 12); CS(13, 14); CS(0, 8); CS(4, 12);
    CS(4, 8); CS(2, 10); CS(6, 14); CS(6, 10); CS(2, 4); CS(6, 8); CS(10, 12); CS(1, 9);
    CS(5, 13); CS(5, 9); CS(3, 11); CS(7, 15); CS(7, 11); CS(3, 5); CS(7, 9); CS(11, 13);
    CS(1, 2); CS(3, 4); CS(5, 6); CS(7, 8); CS(9, 10); CS(11, 12); CS(13, 14);
#undef CS
}

struct Acc {
    double bsum[4];
    uint32_t cpack;     // c[base] in 8-bit fields
    uint64_t wpack;     // w[strand<<2|base] in 8-bit fields
};

// one key of errmod_cal's descending loop (pop_utils.cpp:303-314)
__device__ __forceinline__ void errmod_step(Acc &a, uint32_t key, int n_eff, const double *s_fk,
                                            const double *__restrict__ beta) {
    int q = (int)(key >> 5);                 // already clamped to [4,63] by call_base
    int base = (int)(key & 3);
    int widx = (int)(((key >> 4) & 1) << 2) | base;
    uint32_t c = (a.cpack >> (8 * base)) & 0xFF;
    uint32_t w = (uint32_t)(a.wpack >> (8 * widx)) & 0xFF;
    double term = s_fk[w] * beta[(q << 16) | (n_eff << 8) | (int)c];
    // exactly one accumulator receives the product (x + 0.0 == x for the others is
    // avoided by selecting, to keep the reference's single rounding per addition)
    if (base == 0) a.bsum[0] += term;
    else if (base == 1) a.bsum[1] += term;
    else if (base == 2) a.bsum[2] += term;
    else a.bsum[3] += term;
    a.cpack += 1u << (8 * base);
    a.wpack += 1ULL << (8 * widx);
}

// call_base's per-read part (popbam.cpp:266-286): returns key or 0xFFFFFFFF if filtered
__device__ __forceinline__ uint32_t read_key(uint32_t r, const DevParams &P, int &mapq) {
    int tmp_baseQ = (int)(r & 0xff);
    int baseQ = (P.flag & PBG_F_ILLUMINA) ? (tmp_baseQ > 31 ? tmp_baseQ - 31 : 0) : tmp_baseQ;
    mapq = (int)((r >> 8) & 0xff);
    if (baseQ < P.min_baseQ || mapq < P.min_mapQ) return 0xFFFFFFFFu;
    int b = kNt16Nt4[(r >> 16) & 0xf];
    if (b > 3) return 0xFFFFFFFFu;
    int qq = baseQ < mapq ? baseQ : mapq;
    qq = qq < 4 ? 4 : (qq > 63 ? 63 : qq);
    return (uint32_t)(qq << 5) | (((r >> 20) & 1u) << 4) | (uint32_t)b;
}

// errmod_cal's likelihood block (pop_utils.cpp:316-362) + gl2cns (pop_utils.cpp:66-100);
// returns the consensus word without rms.
__device__ __forceinline__ uint64_t likelihood_gl2cns(const Acc &a, int k, const double *__restrict__ lhet) {
    uint32_t c[4] = {a.cpack & 0xFF, (a.cpack >> 8) & 0xFF, (a.cpack >> 16) & 0xFF, (a.cpack >> 24) & 0xFF};
    float q[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float tmp1 = 0.0f;
        int tmp2 = 0;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            if (kk == j) continue;
            tmp1 = (float)((double)tmp1 + a.bsum[kk]);
            tmp2 += (int)c[kk];
        }
        float v = tmp2 ? tmp1 : 0.0f;
        q[j][j] = v < 0.0f ? 0.0f : v;
#pragma unroll
        for (int kk = j + 1; kk < 4; ++kk) {
            int cjk = (int)(c[j] + c[kk]);
            float t1 = 0.0f;
            int t2 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i == j || i == kk) continue;
                t1 = (float)((double)t1 + a.bsum[i]);
                t2 += (int)c[i];
            }
            double lh = -4.343 * lhet[(cjk << 8) | (int)c[kk]];
            float hv = t2 ? (float)(lh + (double)t1) : (float)lh;
            q[j][kk] = hv < 0.0f ? 0.0f : hv;
        }
    }
    if (k == 0) {  // errmod_cal returns with q zeroed
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int kk = j; kk < 4; ++kk) q[j][kk] = 0.0f;
    }
    float mn = 3.40282347e+38f, mn_next = 3.40282347e+38f;   // FLT_MAX
    uint32_t min_ij = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) {
            float l = q[i][j];
            if (l < mn) {
                min_ij = (uint32_t)(i << 2 | j);
                mn_next = mn;
                mn = l;
            } else if (l < mn_next) {
                mn_next = l;
            }
        }
    uint64_t snpq = (uint64_t)((double)(mn_next - mn) + 0.499) << 32;
    return snpq + ((uint64_t)k << 16) + ((uint64_t)min_ij << 8);
}

// x86-64 double->u64 of NaN gives 0x8000000000000000; rms<<48 then drops it.
__device__ __forceinline__ uint64_t rms_word(int rmsq, int k) {
    float f = (float)rmsq / (float)k;
    double d = (double)__builtin_sqrtf(f) + 0.499;
    uint64_t r = (d != d) ? 0x8000000000000000ULL : (uint64_t)d;
    return r << 48;
}

// Slow path for k > kFastKeys: descending (key, index) selection directly over the reads,
// honouring the n>255 rotate-and-truncate of ks_shuffle (ksort.h:254-262).
__device__ uint64_t call_sample_slow(const uint32_t *rec, int d, int k, const DevParams &P,
                                     const double *s_fk, const DevTables &T) {
    int n_eff = k > 255 ? 255 : k;
    // filtered index range kept: all if k<=255, else [1,255] (rotation drops index 0)
    int lo = k > 255 ? 1 : 0, hi = k > 255 ? 255 : k - 1;
    Acc a;
    a.bsum[0] = a.bsum[1] = a.bsum[2] = a.bsum[3] = 0.0;
    a.cpack = 0;
    a.wpack = 0;
    uint32_t prev_key = 0xFFFFFFFFu;
    int prev_idx = -1;
    for (int step = 0; step < n_eff; ++step) {
        uint32_t best_key = 0;
        int best_idx = -1;
        int fi = 0;
        for (int i = 0; i < d; ++i) {
            int mq;
            uint32_t key = read_key(rec[i], P, mq);
            if (key == 0xFFFFFFFFu) continue;
            int idx = fi++;
            if (idx < lo || idx > hi) continue;
            // candidate must come strictly after prev in (key desc, idx asc) order
            bool after = key < prev_key || (key == prev_key && idx > prev_idx);
            bool better = best_idx < 0 || key > best_key || (key == best_key && idx < best_idx);
            if (after && better) {
                best_key = key;
                best_idx = idx;
            }
        }
        prev_key = best_key;
        prev_idx = best_idx;
        errmod_step(a, best_key, n_eff, s_fk, T.beta);
    }
    return likelihood_gl2cns(a, k, T.lhet);
}

// clean_heterozygotes / segbase / qfilter, per-sample parts (pop_utils.cpp:102-201).
// Returns info byte: bit0 pass, bit1 derived, bits 2-3 allele (for segbase's baseCount).
__device__ __forceinline__ uint32_t site_filters(uint64_t &cb, unsigned char refc, const DevParams &P) {
    unsigned char r = iupac_rev(refc);
    if (!(P.flag & PBG_F_HETEROZYGOTE)) {
        unsigned g = (unsigned)(cb >> 8) & 0xff;
        unsigned a1 = (g >> 2) & 3, a2 = g & 3;
        unsigned sq = (unsigned)(cb >> 32) & 0xffff;
        int64_t d = (int64_t)a2 - (int64_t)a1;
        if (a1 != a2 && (int)sq >= P.min_snpQ) {
            if (a1 == r) cb += (uint64_t)(d * 1024);
            if (a2 == r) cb -= (uint64_t)(d * 256);
        }
        if (a1 != a2 && (int)sq < P.min_snpQ) {
            if (a1 != r) cb += (uint64_t)(d * 1024);
            if (a2 != r) cb -= (uint64_t)(d * 256);
        }
    }
    uint32_t info = 0;
    {
        unsigned g = (unsigned)(cb >> 8) & 0xff;
        unsigned a1 = (g >> 2) & 3, a2 = g & 3;
        unsigned sq = (unsigned)(cb >> 32) & 0xffff;
        // iupac[g] for hom g (a1==a2) is one of A,C,G,T: compare case-sensitively (A.5)
        if (a1 == a2 && iupac_hom(g) != (char)refc) {
            if ((int)sq >= P.min_snpQ) {
                cb |= 2ULL;
                info |= 2u | (a1 << 2);
            } else {
                int64_t d = (int64_t)g - (int64_t)r;     // revert; second step borrows (A.3)
                cb -= (uint64_t)(d * 256);
                cb -= (uint64_t)(d * 1024);
            }
        }
    }
    unsigned rms = (unsigned)(cb >> 48) & 0xffff;
    unsigned nr = (unsigned)(cb >> 16) & 0xffff;
    if ((int)rms >= P.min_rmsQ && (int)nr >= P.min_depth && (int)nr <= P.max_depth) {
        cb |= 1ULL;
        info |= 1u;
    }
    return info;
}

template <int RB>
struct RowW;
template <> struct RowW<2> { using T = uint16_t; };
template <> struct RowW<4> { using T = uint32_t; };
template <> struct RowW<8> { using T = uint64_t; };
template <> struct RowW<16> { using T = ulonglong2; };

template <int RB>
__device__ __forceinline__ void store_row(void *rows, size_t i, uint64_t types, bool counted, bool seg) {
    if constexpr (RB == 16) {
        ulonglong2 v;
        v.x = counted ? types : 0;
        v.y = counted ? ((1ULL << 62) | (seg ? (1ULL << 63) : 0)) : 0;
        reinterpret_cast<ulonglong2 *>(rows)[i] = v;
    } else {
        using T = typename RowW<RB>::T;
        constexpr int W = RB * 8;
        uint64_t v = counted ? (types | (1ULL << (W - 2)) | (seg ? (1ULL << (W - 1)) : 0)) : 0;
        reinterpret_cast<T *>(rows)[i] = (T)v;
    }
}

}  // namespace

// Dynamic LDS layout (bytes): s_fk[256] f64 | s_dep[64n] u16 | s_off[64n+1] u32 |
//                             s_info[64n] u8 | s_reads[cap] u32
template <int RB>
__global__ __launch_bounds__(kBlockThreads) void call_sites_kernel(
    DevParams P, DevTables T, uint32_t n_sites, const uint8_t *__restrict__ ref,
    const uint16_t *__restrict__ depth, const uint64_t *__restrict__ block_off,
    const uint32_t *__restrict__ reads, uint32_t cap, void *__restrict__ rows,
    uint64_t *__restrict__ cb_out, int *__restrict__ err) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int n = P.n;
    const int tid = threadIdx.x;
    const uint32_t blk = blockIdx.x;
    const uint32_t site0 = blk * kSiteBlock;
    const int nsb = (int)min((uint32_t)kSiteBlock, n_sites - site0);
    const int ntask = nsb * n;

    double *s_fk = reinterpret_cast<double *>(smem);
    uint16_t *s_dep = reinterpret_cast<uint16_t *>(s_fk + 256);
    uint32_t *s_off = reinterpret_cast<uint32_t *>(s_dep + ((kSiteBlock * n + 1) & ~1));
    unsigned char *s_info = reinterpret_cast<unsigned char *>(s_off + kSiteBlock * n + 1);
    uint32_t *s_reads = reinterpret_cast<uint32_t *>(
        (reinterpret_cast<uintptr_t>(s_info + kSiteBlock * n) + 15) & ~uintptr_t(15));
    __shared__ uint32_t s_wsum[kBlockThreads / 64];

    for (int i = tid; i < 256; i += kBlockThreads) s_fk[i] = T.fk[i];
    const uint16_t *gdep = depth + (size_t)site0 * n;
    for (int i = tid; i < ntask; i += kBlockThreads) s_dep[i] = gdep[i];
    __syncthreads();

    // exclusive scan of the block's depths -> per-task read offsets
    constexpr int PER = (kSiteBlock * PBG_MAX_SAMPLES + kBlockThreads - 1) / kBlockThreads;  // 16
    uint32_t loc[PER];
    uint32_t run = 0;
    const int t0 = tid * PER;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        int t = t0 + j;
        uint32_t v = t < ntask ? s_dep[t] : 0;
        loc[j] = run;
        run += v;
    }
    // wave64 inclusive scan of `run`
    const int lane = tid & 63, wv = tid >> 6;
    uint32_t incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wv; ++w) wbase += s_wsum[w];
    const uint32_t excl = wbase + incl - run;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        int t = t0 + j;
        if (t < ntask) s_off[t] = excl + loc[j];
    }
    if (tid == kBlockThreads - 1) s_off[ntask] = excl + run;
    __syncthreads();

    const uint64_t gbase = block_off[blk];
    const uint32_t total = s_off[ntask];
    if (block_off[blk + 1] - gbase != total) {   // inconsistent batch: never read past it
        if (tid == 0) atomicOr(err, 1);
        if (tid < nsb) store_row<RB>(rows, (size_t)site0 + tid, 0, false, false);
        return;
    }

    // stage the block's reads: LDS index i <-> global index (gbase & ~3) + i
    const uint64_t a0 = gbase & ~uint64_t(3);
    const uint32_t shift = (uint32_t)(gbase - a0);
    const bool staged = total + shift <= cap;
    if (staged && total) {
        const uint64_t gend = gbase + total;
        const uint64_t va = (gbase + 3) & ~uint64_t(3), vb = gend & ~uint64_t(3);
        if (va < vb) {
            const uint4 *src = reinterpret_cast<const uint4 *>(reads + va);
            uint4 *dst = reinterpret_cast<uint4 *>(s_reads + (va - a0));
            const uint32_t nv = (uint32_t)((vb - va) >> 2);
            for (uint32_t i = tid; i < nv; i += kBlockThreads) dst[i] = src[i];
        }
        for (uint64_t g = gbase + tid; g < va && g < gend; g += kBlockThreads) s_reads[g - a0] = reads[g];
        for (uint64_t g = (vb > va ? vb : va) + tid; g < gend; g += kBlockThreads) s_reads[g - a0] = reads[g];
    }
    __syncthreads();

    for (int t = tid; t < ntask; t += kBlockThreads) {
        const int sl = t / n;
        const uint32_t site = site0 + sl;
        const unsigned char refc = ref[site];
        uint64_t cb = 0;
        uint32_t info = 0;
        if (!(refc & 0x80)) {
            const int d = s_dep[t];
            if (d > 0) {
                const uint32_t *rec = staged ? (s_reads + shift + s_off[t]) : (reads + gbase + s_off[t]);
                // pass 1: filter, collect up to kFastKeys keys, count k, sum mapQ^2
                uint32_t key[kFastKeys];
#pragma unroll
                for (int j = 0; j < kFastKeys; ++j) key[j] = 0;
                int k = 0, rmsq = 0;
                for (int i = 0; i < d; ++i) {
                    int mq;
                    uint32_t kk = read_key(rec[i], P, mq);
                    if (kk == 0xFFFFFFFFu) continue;
#pragma unroll
                    for (int j = 0; j < kFastKeys; ++j)
                        if (j == k) key[j] = kk;
                    ++k;
                    rmsq += mq * mq;
                }
                if (k <= kFastKeys) {
                    sort16_desc(key);
                    Acc a;
                    a.bsum[0] = a.bsum[1] = a.bsum[2] = a.bsum[3] = 0.0;
                    a.cpack = 0;
                    a.wpack = 0;
#pragma unroll
                    for (int j = 0; j < kFastKeys; ++j)
                        if (j < k) errmod_step(a, key[j], k, s_fk, T.beta);
                    cb = likelihood_gl2cns(a, k, T.lhet);
                } else {
                    cb = call_sample_slow(rec, d, k, P, s_fk, T);
                }
                cb |= rms_word(rmsq, k);
            }
            info = site_filters(cb, refc, P) | 0x10u;   // bit4: position called back
        }
        s_info[t] = (unsigned char)info;
        if (cb_out) cb_out[(size_t)site0 * n + t] = cb;
    }
    __syncthreads();

    // fold samples per position: segbase's fq (pop_utils.cpp:154-167), qfilter coverage,
    // cal_site_type (popbam.cpp:173-184)
    if (tid < nsb) {
        const unsigned char *inf = s_info + tid * n;
        int cnt[4] = {0, 0, 0, 0};
        int pass = 0;
        uint64_t types = 0;
        bool called = (inf[0] & 0x10u) != 0;
        for (int j = 0; j < n; ++j) {
            uint32_t v = inf[j];
            pass += (int)(v & 1u);
            if (v & 2u) {
                int al = (int)((v >> 2) & 3u);
                cnt[0] += al == 0; cnt[1] += al == 1; cnt[2] += al == 2; cnt[3] += al == 3;
            }
            if ((v & 3u) == 3u) types |= 1ULL << j;
        }
        int nz = 0, kk = 0;
        for (int i = 0; i < 4; ++i)
            if (cnt[i] > 0) { ++nz; kk = i; }
        int fq = nz > 1 ? -1 : cnt[kk];
        bool counted = called && pass == n;
        store_row<RB>(rows, (size_t)site0 + tid, types, counted, counted && fq > 0);
    }
}

// ------------------------------------------------------------------ synthetic pileup
__global__ __launch_bounds__(kBlockThreads) void synth_depth_kernel(uint64_t seed, int mean_depth, int n,
                                                                    uint32_t n_sites, uint8_t *ref,
                                                                    uint16_t *depth, uint64_t *block_tot) {
    __shared__ uint32_t s_sum[kBlockThreads / 64];
    const uint32_t site0 = blockIdx.x * kSiteBlock;
    const int nsb = (int)min((uint32_t)kSiteBlock, n_sites - site0);
    uint32_t acc = 0;
    for (int t = threadIdx.x; t < nsb * n; t += kBlockThreads) {
        int sl = t / n, s = t - sl * n;
        SynthSite ss = synth_site(seed, site0 + sl);
        int d = synth_depth(synth_sample_hash(ss, s), mean_depth);
        depth[(size_t)site0 * n + t] = (uint16_t)d;
        acc += (uint32_t)d;
        if (s == 0) ref[site0 + sl] = synth_ref_char(ss);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kBlockThreads / 64; ++w) t += s_sum[w];
        block_tot[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBlockThreads) void synth_reads_kernel(uint64_t seed, int mean_depth, int n,
                                                                    uint32_t n_sites, const uint16_t *depth,
                                                                    const uint64_t *block_off, uint32_t *reads) {
    // one thread per (position, sample): offsets by a serial scan of the block's depths in LDS
    extern __shared__ uint32_t s_off2[];
    const uint32_t site0 = blockIdx.x * kSiteBlock;
    const int nsb = (int)min((uint32_t)kSiteBlock, n_sites - site0);
    const int ntask = nsb * n;
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int t = 0; t < ntask; ++t) {
            s_off2[t] = run;
            run += depth[(size_t)site0 * n + t];
        }
    }
    __syncthreads();
    const uint64_t base = block_off[blockIdx.x];
    for (int t = threadIdx.x; t < ntask; t += kBlockThreads) {
        int sl = t / n, s = t - sl * n;
        SynthSite ss = synth_site(seed, site0 + sl);
        uint64_t hs = synth_sample_hash(ss, s);
        int d = depth[(size_t)site0 * n + t];
        uint32_t *out = reads + base + s_off2[t];
        for (int r = 0; r < d; ++r) out[r] = synth_read(ss, hs, r);
    }
}

template __global__ void call_sites_kernel<2>(DevParams, DevTables, uint32_t, const uint8_t *, const uint16_t *,
                                              const uint64_t *, const uint32_t *, uint32_t, void *, uint64_t *, int *);
template __global__ void call_sites_kernel<4>(DevParams, DevTables, uint32_t, const uint8_t *, const uint16_t *,
                                              const uint64_t *, const uint32_t *, uint32_t, void *, uint64_t *, int *);
template __global__ void call_sites_kernel<8>(DevParams, DevTables, uint32_t, const uint8_t *, const uint16_t *,
                                              const uint64_t *, const uint32_t *, uint32_t, void *, uint64_t *, int *);
template __global__ void call_sites_kernel<16>(DevParams, DevTables, uint32_t, const uint8_t *, const uint16_t *,
                                               const uint64_t *, const uint32_t *, uint32_t, void *, uint64_t *, int *);

}  // namespace pbg

namespace pbg {

size_t call_sites_lds_bytes(int n, uint32_t cap) {
    size_t b = 256 * 8;                                   // s_fk
    b += (size_t)((kSiteBlock * n + 1) & ~1) * 2;         // s_dep
    b += (size_t)(kSiteBlock * n + 1) * 4;                // s_off
    b += (size_t)kSiteBlock * n;                          // s_info
    b = (b + 15) & ~size_t(15);
    b += (size_t)cap * 4 + 16;                            // s_reads
    return b;
}

hipError_t launch_call_sites(int rb, const DevParams &P, const DevTables &T, uint32_t n_sites, const uint8_t *ref,
                             const uint16_t *depth, const uint64_t *block_off, const uint32_t *reads, uint32_t cap,
                             void *rows, uint64_t *cb, int *err, hipStream_t stream) {
    const uint32_t nblk = (n_sites + kSiteBlock - 1) / kSiteBlock;
    if (nblk == 0) return hipSuccess;
    const size_t lds = call_sites_lds_bytes(P.n, cap);
    dim3 g(nblk), b(kBlockThreads);
    switch (rb) {
        case 2: hipLaunchKernelGGL(call_sites_kernel<2>, g, b, lds, stream, P, T, n_sites, ref, depth, block_off, reads, cap, rows, cb, err); break;
        case 4: hipLaunchKernelGGL(call_sites_kernel<4>, g, b, lds, stream, P, T, n_sites, ref, depth, block_off, reads, cap, rows, cb, err); break;
        case 8: hipLaunchKernelGGL(call_sites_kernel<8>, g, b, lds, stream, P, T, n_sites, ref, depth, block_off, reads, cap, rows, cb, err); break;
        default: hipLaunchKernelGGL(call_sites_kernel<16>, g, b, lds, stream, P, T, n_sites, ref, depth, block_off, reads, cap, rows, cb, err); break;
    }
    return hipGetLastError();
}

hipError_t launch_synth_depth(uint64_t seed, int mean_depth, int n, uint32_t n_sites, uint8_t *ref, uint16_t *depth,
                              uint64_t *block_tot, hipStream_t stream) {
    const uint32_t nblk = (n_sites + kSiteBlock - 1) / kSiteBlock;
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_depth_kernel, dim3(nblk), dim3(kBlockThreads), 0, stream, seed, mean_depth, n, n_sites, ref,
                       depth, block_tot);
    return hipGetLastError();
}

hipError_t launch_synth_reads(uint64_t seed, int mean_depth, int n, uint32_t n_sites, const uint16_t *depth,
                              const uint64_t *block_off, uint32_t *reads, hipStream_t stream) {
    const uint32_t nblk = (n_sites + kSiteBlock - 1) / kSiteBlock;
    if (nblk == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_reads_kernel, dim3(nblk), dim3(kBlockThreads), (size_t)kSiteBlock * n * 4, stream, seed,
                       mean_depth, n, n_sites, depth, block_off, reads);
    return hipGetLastError();
}

}  // namespace pbg
