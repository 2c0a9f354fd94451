// pbg_common.h -- types shared by the host orchestration and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/popbam_gpu.h"
#define PBG_HD __host__ __device__
#include "pbg_key.h"

// Experiment switches (timing variants; PBG_SLOW_NONET and PBG_ZNS_EXP even give wrong results)
// compile only in a variant build that says so: tools/variant.sh adds -DPBG_EXPERIMENT=1.  The
// product build (popbam_csrc/Makefile) cannot take one by accident, and every translation unit
// records its build kind for pbg_build_info() (product / bounds / experiment).
#if !defined(PBG_EXPERIMENT)
#if defined(PBG_SLOW_NONET) || defined(PBG_ZNS_EXP) || defined(PBG_ZNS_SORT) || defined(PBG_ZNS_PRIO) || \
    defined(PBG_SCAN_WIDE_PASS) || defined(PBG_CALL_WAVES_PER_SIMD) || defined(PBG_SLOW_WG_PER_CU) ||      \
    defined(PBG_WIN_AHEAD) || defined(PBG_FAST_MAX) || defined(PBG_SYNTH_EXP) || defined(PBG_SCAN_EXP) || \
    defined(PBG_SCAN_LDS_PAD) || defined(PBG_ZNS_GROUPS)
#error "an experiment switch is defined: build variants with tools/variant.sh (-DPBG_EXPERIMENT=1)"
#endif
#define PBG_BUILD_KIND (PBG_BOUNDS_KIND)
#else
#define PBG_BUILD_KIND 2
#endif
#ifdef PBG_BOUNDS
#define PBG_BOUNDS_KIND 1
#else
#define PBG_BOUNDS_KIND 0
#endif

namespace pbg {

constexpr int kBlockThreads = 256;     // 4 wave64 per workgroup
constexpr int kSiteBlock = PBG_SITE_BLOCK;

// reference-only tasks (every key on the reference base) are settled by the scan kernel up to
// this many keys (16 or 32)
#ifndef PBG_FAST_MAX
#define PBG_FAST_MAX 32
#endif
// Parameters passed by value to the kernels (kernarg segment).
struct DevParams {
    int32_t n, npops;
    uint64_t pop_mask[PBG_MAX_POPS];
    uint64_t pop_mask_hi[PBG_MAX_POPS];   // samples 64..125 (n > 64)
    int32_t pop_n[PBG_MAX_POPS];
    int32_t min_depth, max_depth, min_rmsQ, min_snpQ, min_mapQ, min_baseQ;
    uint32_t flag;
    int32_t k16;          // k[] is u16 (max_depth > 255), else u8
    int32_t sfs_stride;   // largest population + 1 (pbg_window_out.sfs_bins row)
    int32_t pop_nmax;     // members of the largest population (calc_nhaps' local indices stay below it)
    int32_t pops_ordered; // every member of population a has a smaller id than every member of b > a
    int8_t sample_pop[PBG_MAX_SAMPLES];   // population of each sample (-1: none); masks are disjoint
    uint8_t pop_member[PBG_MAX_SAMPLES];  // the samples of population 0, then 1, ... (ascending within one)
    int16_t pop_start[PBG_MAX_POPS + 1];  // population i's samples: pop_member[pop_start[i], pop_start[i+1])
    // qfilter of a reference-only sample with k = d keys (call_scan_kernel): it passes iff
    // sum mapQ^2 >= rms_thr[d].  rms = (unsigned)(sqrtf((float)rmsq / d) + 0.499) is monotone in
    // rmsq, so "rms >= min_rmsQ && min_depth <= d <= max_depth" is one threshold per d, found on
    // the host with the same IEEE float division and square root (rms_threshold, api.cpp).
    uint32_t rms_thr[PBG_FAST_MAX + 1];
    // qfilter's rms test alone, for k = 0..16 keys: rms >= min_rmsQ iff sum mapQ^2 >= rmsq_thr[k]
    // (k = 0: rms is 0 -- the x86 NaN conversion -- so 0 when min_rmsQ <= 0, else never)
    uint32_t rmsq_thr[17];
    // uniform tasks (call_scan_kernel's list pass, uniform_ref): d = 1..16 keys of one base m,
    // uni[d * 3 + cls] (cls 0: m = 0, 1: m = 3, 2: m = 1 or 2) = the smallest q_min at which the
    // strand-free bound fk_prefix[d] * min_{q' >= q_min, c <= d-1} beta[q'][d][c] clears the
    // smallest het m/x value (the margins of one_error_ref; 255: never) | that value's snpq << 8
    uint32_t uni[17 * 3];
};

// Host-built tables resident in HBM for the lifetime of a context.
struct DevTables {
    const double *fk;     // [256]            fk[n]   (pop_utils.cpp:216-219)
    const double *beta;   // [64*256*256]     beta[q<<16|n<<8|k] (pop_utils.cpp:230-245)
    const double *lhet;   // [256*256]        lhet[n<<8|k] (pop_utils.cpp:248-251)
    // fk[w] * beta[q<<16|n<<8|c] for the register path (n <= 16 keys, c, w < 16), indexed
    // fbeta_index(q, n, c, w).  The product is the one IEEE double multiply errmod_cal does
    // per key (pop_utils.cpp:311), so the table value is bit-identical to it.
    const double *fbeta;  // [64*17*16*16]
    // one-error bound (call_slow_kernel): [0, 17) fk_prefix[m] = sum_{w < m} fk[w]; then
    // [17 + (q - 4) * 17 + d] = min over q' in [q, 63], c in [0, d - 2] of beta[q'<<16|d<<8|c]
    // (q 4..63, d 3..16): with m0 / m1 reference-base keys per strand, all of quality >= q,
    // errmod_cal's bsum of that base is >= (fk_prefix[m0] + fk_prefix[m1]) * bmin[q][d]
    const double *lb;     // [17 + 60 * 17]
    // one-error tables in compact form (the scan kernel reads them through L1 / L2):
    // [0, 60 * 17) beta[q<<16|d<<8|0] at (q - 4) * 17 + d; then [60 * 17, 60 * 17 + 17 * 17)
    // lhet[n<<8|k] at 60 * 17 + n * 17 + k (n, k <= 16)
    const double *oe;     // [kOeSize]
    // call_scan_kernel's one-error tables as one image its workgroups copy to LDS (ScanTab, n <= 12):
    // fpe[(q - 4) * 14 + d - 3] = (float)(fk[0] * beta[q<<16|d<<8|0]) (the one double multiply and
    // narrowing one_error_ref does); lq[((q - 4) >> 2) * 14 + d - 3] = lb[17 + (q - 4) * 17 + d] at the
    // level's lowest q, rounded down to float (a lower bound of the bound: the test stays exact,
    // a few more tasks queue); lh[(d - 3) * 4 + i] = -4.343 * lhet of {[d][d-1], [d][1], [d-1][0],
    // [d-1][d-1]} (the double products one_error_ref forms); pre[m] = lb[m] (fk prefix sums)
    const uint4 *scantab;
    const double *a1, *a2, *e1, *e2;          // Tajima/Fay-Wu constants (pop_sfs.cpp:511-571)
    const double *r2;     // concatenated per-population r^2 tables, see r2_off
    int32_t r2_off[PBG_MAX_POPS];             // offset of population p's (n_p+1)^3 table
};

constexpr int kLbSize = 17 + 60 * 17;
struct ScanTab {
    float fpe[60 * 14];
    float lq[15 * 14];
    double lh[14 * 4];
    double pre[17];
};
static_assert(sizeof(ScanTab) % 16 == 0, "ScanTab is copied as uint4");
constexpr int kScanTabVec = (int)(sizeof(ScanTab) / 16);
constexpr int kOeSize = 60 * 17 + 17 * 17;
constexpr int kFbetaN = 17;   // n in [0, 16]
__host__ __device__ inline uint32_t fbeta_index(uint32_t q, uint32_t n, uint32_t c, uint32_t w) {
    return ((q * kFbetaN + n) << 8) | (c << 4) | w;
}
constexpr size_t kFbetaSize = 64u * kFbetaN * 256u;

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Synthetic pileup (benchmark workload): site hash keyed on (seed, contig,
// pos); contig 0 hashes the position alone.
struct SynthSite {
    uint64_t h;
    int ref_idx, alt, snp;
    uint32_t f16;
};
// the site's fields from its hash (kernels hash each position once and share it across samples)
__host__ __device__ inline SynthSite synth_site_h(uint64_t h) {
    SynthSite s;
    s.h = h;
    s.ref_idx = (int)(s.h & 3);
    s.snp = ((s.h >> 2) & 0x3FF) < 12;          // theta ~ 0.012
    s.alt = (s.ref_idx + 1 + (int)((((s.h >> 12) & 0xFFFFu) * 3u) >> 16)) & 3;   // 1..3 steps away
    s.f16 = (uint32_t)((s.h >> 16) & 0xFFFF);   // derived allele frequency
    return s;
}
__host__ __device__ inline uint64_t synth_site_hash(uint64_t seed, int contig, uint64_t pos) {
    return splitmix64(seed ^ splitmix64(pos ^ ((uint64_t)(uint32_t)contig << 40)));
}
__host__ __device__ inline SynthSite synth_site(uint64_t seed, int contig, uint64_t pos) {
    SynthSite s;
    s.h = synth_site_hash(seed, contig, pos);
    s.ref_idx = (int)(s.h & 3);
    s.snp = ((s.h >> 2) & 0x3FF) < 12;          // theta ~ 0.012
    s.alt = (s.ref_idx + 1 + (int)((((s.h >> 12) & 0xFFFFu) * 3u) >> 16)) & 3;   // 1..3 steps away
    s.f16 = (uint32_t)((s.h >> 16) & 0xFFFF);   // derived allele frequency
    return s;
}
// 32-bit finaliser (lowbias32): two 32-bit multiplies, ~4x cheaper than splitmix64's 64-bit ones
__host__ __device__ inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
// per (position, sample): 64 bits from the two halves of the site hash, each keyed on the sample
// by a 24-bit constant (the multiply is a full-rate v_mul_u32_u24: (sample + 1) * K < 2^31)
__host__ __device__ inline uint64_t synth_sample_hash(const SynthSite &s, int sample) {
    const uint32_t m = (uint32_t)(sample + 1);
    const uint32_t lo = mix32((uint32_t)s.h ^ (m * 0xD1B54Bu));
    const uint32_t hi = mix32((uint32_t)(s.h >> 32) ^ (m * 0x9E3779u));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__host__ __device__ inline int synth_depth(uint64_t hs, int mean_depth) {
    // binomial(2D, 1/2): popcount of 2D random bits (mean D), D <= 32
    const int nb = 2 * mean_depth;
    const uint32_t b0 = mix32((uint32_t)hs ^ 0x5851F42Du);
    if (nb <= 32) return __builtin_popcount(b0 & (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)));
    const uint32_t b1 = mix32((uint32_t)(hs >> 32) ^ 0x4C957F2Du);
    const uint64_t m = nb >= 64 ? ~0ULL : ((1ULL << nb) - 1);
    return __builtin_popcountll(((uint64_t)b0 | ((uint64_t)b1 << 32)) & m);
}
// The per-read draws come from a table of read templates (kTmplN entries + a tail, 2 MB as u16).
// Positions come in spans of 16,384 (absolute position >> 14); a span draws its windows from one
// page of the table, kTmplPage entries at synth_tmpl_page(seed, contig, pos), and a position's
// window starts at a random multiple of 64 in that page (synth_tmpl_base: 64 starts a page, 16 K
// over the table, as many as a window anywhere in the table would have).  Its samples read
// interleaved 8-entry chunks of the window: read r of sample s (of n) is entry
// base + 8 (s + n (r >> 3)) + (r & 7) (synth_tmpl_index).  Distinct samples read distinct
// entries; chunk c of a position's consecutive samples is one contiguous run (coalesced loads);
// and a workgroup of consecutive positions finds every read it needs in one page plus the
// window's reach, which fits LDS (r05: the keys kernel reads its templates from LDS, not through
// the vector cache it writes 16 GB a chunk through).  Entry i: bq << 5 | strand << 4 | hap << 2,
// drawn from 32 random bits hr_i: haplotype (bit 0), baseQ 20..40 (bits 16-31), strand (bit 8 ^
// bit 17).  Fixed-point ranges, no division.  Sequencing errors are the task's own
// (synth_errors), not the template's: positions that share a page would otherwise share its
// errors, and the spurious segregating sites two errors in one sample make would cluster by
// span (a 10 kb window's count: sd 120 against 16 with the errors drawn per task).
constexpr uint32_t kTmplN = 1u << 20;
constexpr uint32_t kTmplPage = 4096;            // entries whose 64-entry steps a page's windows start at
constexpr int kTmplSpanShift = 14;              // positions share a page in spans of 16,384
constexpr uint32_t kTmplSize = kTmplN + 8192;   // a window reaches base + 8 (125 + 126 * 7) + 8 (64 reads, 126 samples)
__host__ __device__ inline uint32_t synth_tmpl_seed(uint64_t seed) {
    return (uint32_t)splitmix64(seed ^ 0x6A09E667F3BCC909ULL);
}
__host__ __device__ inline uint32_t synth_tmpl_entry(uint32_t tseed, uint32_t i) {
    const uint32_t hr = mix32(tseed ^ (0x9E3779B9u * (i + 1u)));
    const uint32_t bq = 20u + ((((hr >> 16) & 0xFFFFu) * 21u) >> 16);
    const uint32_t strand = ((hr >> 8) ^ (hr >> 17)) & 1u;
    return (bq << 5) | (strand << 4) | ((hr & 1u) << 2);
}
// the page of a position's span: a multiple of kTmplPage in [0, kTmplN)
__host__ __device__ inline uint32_t synth_tmpl_page(uint64_t seed, int contig, uint64_t pos) {
    const uint64_t span = (pos >> kTmplSpanShift) | ((uint64_t)(uint32_t)contig << 40);
    return (uint32_t)(splitmix64(seed ^ 0x243F6A8885A308D3ULL ^ span) & (kTmplN / kTmplPage - 1)) * kTmplPage;
}
// a position's template window: its span's page + 64 x (bits 32..37 of its site hash; the site
// fields use bits 0..31)
__host__ __device__ inline uint32_t synth_tmpl_base(uint64_t h, uint32_t page) {
    return page + (uint32_t)((h >> 32) & (kTmplPage / 64 - 1)) * 64u;
}
// template entry of read r of sample s (of n) at a position with window base
__host__ __device__ inline uint32_t synth_tmpl_index(uint32_t base, uint32_t n, uint32_t s, uint32_t r) {
    return base + 8u * (s + n * (r >> 3)) + (r & 7u);
}
// the task's two haplotype alleles a0 | a1 << 2
__host__ __device__ inline uint32_t synth_alleles(const SynthSite &s, uint64_t hs) {
    const int a0 = (s.snp && (uint32_t)(hs & 0xFFFF) < s.f16) ? s.alt : s.ref_idx;
    const int a1 = (s.snp && (uint32_t)((hs >> 16) & 0xFFFF) < s.f16) ? s.alt : s.ref_idx;
    return (uint32_t)(a0 | (a1 << 2));
}
// A task's sequencing errors: at most two of its d reads (d <= 64), P(one) = d/128 (1 - (d-1)/128),
// P(two) = d (d - 1) / 32768 (1 - (d-2)/128) -- the binomial's first two terms at 1/128 a read, to
// first order -- at distinct
// reads j1, j2, each read's base moved e1, e2 in 1..3 steps (weights 3/8, 3/8, 2/8), all from one
// hash of the sample hash's lower half.
struct SynthErr {
    uint32_t ne, j1, j2, e1, e2;
};
__host__ __device__ inline SynthErr synth_errors(uint32_t hs_lo, uint32_t d) {
    const uint32_t eh = mix32(hs_lo ^ 0x2545F491u);
    const uint32_t u = eh & 0x3FFFu;                                  // in 1 / 16384
    const uint32_t dd1 = d * (d > 0u ? d - 1u : 0u);
    const uint32_t p2 = (dd1 * (130u - d)) >> 8, p1 = (d << 7) - dd1;
    SynthErr e;
    e.ne = u < p2 ? 2u : (u < p2 + p1 ? 1u : 0u);
    e.j1 = (((eh >> 14) & 63u) * d) >> 6;
    uint32_t j2 = e.j1 + 1u + (d > 1u ? (((eh >> 20) & 63u) * (d - 1u)) >> 6 : 0u);
    e.j2 = j2 >= d ? j2 - d : j2;
    e.e1 = 1u + ((((eh >> 26) & 7u) * 3u) >> 3);
    e.e2 = 1u + ((((eh >> 29) & 7u) * 3u) >> 3);
    return e;
}
// the error base offset of read r (0: none)
__host__ __device__ inline uint32_t synth_err_off(const SynthErr &e, uint32_t r) {
    return (e.ne >= 1u && r == e.j1 ? e.e1 : 0u) + (e.ne >= 2u && r == e.j2 ? e.e2 : 0u);
}
// raw read word (bits 0-7 baseQ, 8-15 mapQ 60, 16-19 nt16 base, 20 strand) of a template entry
// with the read's error offset in bits 0-1 (the entry's own are zero)
__host__ __device__ inline uint32_t synth_tmpl_read(uint32_t ent, uint32_t alv) {
    const uint32_t base = (((alv >> (2u * ((ent >> 2) & 1u))) & 3u) + (ent & 3u)) & 3u;
    return (ent >> 5) | (60u << 8) | ((1u << base) << 16) | (((ent >> 4) & 1u) << 20);
}
// read r of sample `sample` (of n, depth d) at a site whose span's page is `page`
__host__ __device__ inline uint32_t synth_read(const SynthSite &s, uint64_t hs, uint32_t page, int n, int sample, int d,
                                               int r, uint32_t tseed) {
    const uint32_t ent = synth_tmpl_entry(tseed, synth_tmpl_index(synth_tmpl_base(s.h, page), (uint32_t)n,
                                                                   (uint32_t)sample, (uint32_t)r));
    return synth_tmpl_read(ent | synth_err_off(synth_errors((uint32_t)hs, (uint32_t)d), (uint32_t)r), synth_alleles(s, hs));
}
// every synthetic read survives call_base's filters: baseQ 20..40 (no Illumina offset), mapQ 60,
// one-hot A/C/G/T bases
__host__ __device__ inline bool synth_all_pass(uint32_t min_baseQ, uint32_t min_mapQ, bool illumina) {
    return !illumina && min_baseQ <= 20u && min_mapQ <= 60u;
}
__host__ __device__ inline uint8_t synth_ref_char(const SynthSite &s) { return (uint8_t)"ACGT"[s.ref_idx]; }

constexpr int kSegCap = 256;         // segregating rows kept in LDS per window (beyond: workspace), at most
constexpr int kVarCap = 256;         // ZnS variable-site list kept in LDS per population

// Dynamic LDS of window_stats_kernel (one wave per window): byte offsets of its arrays, sized
// by the host for the sample / population counts and the statistics asked for.
struct WinLds {
    uint32_t seg, var, plane, diff, acc, amin, bins, rbuf, r2, bytes;
    int32_t segcap;     // segregating rows kept in LDS (a multiple of 64, <= kSegCap; beyond: workspace)
    int32_t planecap;   // bitplane words in LDS (n * segcap / 64)
    int32_t r2lds;      // doubles of the r^2 tables copied to LDS (0: read from HBM / L2)
};
// diff: one bit per sample pair (differ / not), for calc_nhaps
WinLds stats_lds_layout(int n, int np, int sfs_stride, uint32_t stats, int r2_total, int mask_words, int segcap);

struct StatsArgs {
    uint32_t stats;
    int32_t min_freq, outidx, jc;
    const pbg_window *wins;
    // Statistics workspace: a pool the windows that need it take slices of with one atomic add
    // (windows with more than kSegCap segregating rows, the omega / Wall lists, the ZnS lists);
    // an exhausted pool sets err bit 4 (pbg_check -> PBG_E_RANGE).
    uint64_t *pool;
    uint64_t pool_cap;                    // u64 words
    unsigned long long *pool_used;        // [1] words taken, zeroed per call
    int *err;
    uint64_t *win_off;                    // [2*n_win] pool offsets: seg rows, omega / Wall lists
    uint64_t *zoff;                       // [n_win*npops] offset of each ZnS chain's list (pool or zlist)
    // ZnS lists at fixed places when the window lengths allow it (zstride > 0): window w,
    // population i at zlist + w * zstride + i * (zstride / npops); else bump-allocated in the pool
    uint64_t *zlist;
    uint64_t zstride;                     // u64 words per window
    int32_t *seg_count;                   // [n_win] segregating rows
    int32_t *var_count;                   // [n_win*npops] ZnS: rows variable within the population
    int32_t *ld_ns;                       // [n_win*npops] ZnS: the reference's num_snps
    pbg_window_out out;
    WinLds lds;
    // PBG_BOUNDS store checks: pool / ZnS-list stores must fall in the first len / pool_div
    // words of the slice they belong to (1; 2 in the PBG_BOUNDS_SELFTEST=pool positive control)
    uint32_t pool_div;
};
#define PBG_POOL_OK(A, idx, lo, len) PBG_STORE_OK((A).err, (idx) - (lo), (len) / (A).pool_div, len, ::pbg::kErrPool)

// Samples deeper than the register sort width (16 reads) are finished outside the main call
// kernel: it queues them as tasks (lane-per-task kernel), parks the position's other per-sample
// info bytes in `info` ([n_sites * n], written only for such positions) and queues the
// position for a final fold.  A task that does not fit in the queue is computed in place.
struct DeepTask {
    uint32_t site;
    uint32_t sd;        // sample | k << 8
    uint64_t off;       // index in keys[] of the task's first key
};
struct DeepBufs {
    uint32_t *sites;    // [n_sites] positions with a queued task
    DeepTask *tasks;    // [task_cap]
    uint8_t *info;      // [n_sites * n]
    uint32_t *count;    // [0] positions, [1] tasks (may exceed task_cap: computed in place),
                        // [2] rows-only pipeline: blocks listed for the overflow kernel,
                        // [3] rows-only pipeline: deep tasks appended to `tasks` (dense list)
    uint32_t task_cap;
    // rows-only pipeline: block b owns queue records raw[b*blk_cap, (b+1)*blk_cap) for the tasks
    // with at most 16 reads the scan could not settle (blk_cnt[b] of them); tasks with more reads
    // are a dense list tasks[0, count[3]) (at most task_cap)
    uint32_t *blk_cnt;
    uint32_t blk_cap;
    uint64_t *pend;     // rows-only pipeline: per block, the positions whose row waits for a queued task
    uint4 *raw;         // [nblk*blk_cap*3] 48-byte queue records {site, sample | k << 8, sum mapQ^2,
                        // reference byte} + the task's 16 keys (0 past k): all call_slow_kernel reads
    // PBG_BOUNDS store checks (unused by the product build): each array's allocated length
    // (elements) and the length the checks allow -- equal, except in a PBG_BOUNDS_SELFTEST mode,
    // which halves one of them so correct kernels trip that class's check (api.cpp)
    uint64_t raw_n, raw_chk;       // uint4 entries of raw
    uint64_t info_n, info_chk;     // bytes of info
    uint32_t tasks_n, tasks_chk;   // entries of tasks
    uint32_t blk_n, blk_chk;       // entries of blk_cnt / pend
    uint32_t sites_n, sites_chk;   // entries of sites
    uint32_t rows_div;             // rows the checks allow = n_sites / rows_div (1; 2 in the rows self-test)
    uint32_t words_div;            // consensus words allowed = n_sites * n / words_div
};
#ifndef PBG_QGROUP
#define PBG_QGROUP 16
#endif
constexpr int kQueueGroup = PBG_QGROUP;   // blocks per wave in the queue kernels

// A device pileup batch as the kernels see it (pbg_pileup with the k width resolved).
struct Batch {
    uint32_t n_sites;
    const uint8_t *ref;
    const void *k;                 // u8 or u16 (DevParams::k16)
    const uint32_t *rmsq;
    const uint64_t *block_off;
    const uint16_t *keys;
    int *err;                      // the context's error word (PBG_BOUNDS checks)
    // the batch has long runs of a lower-case / N reference (the host saw them): the scan then
    // settles its list mid-block instead of sending what overflows it to call_overflow_kernel
    int masked;
    // compact pieces (pbg_stream_push_compact): rmsq bit 31 flags a reference-only task whose keys
    // the batch leaves out; block_off counts the keys present
    int compact;
    // PBG_BOUNDS builds only: keys the checks take off the end of the batch's range (the
    // positive control, PBG_BOUNDS_SELFTEST=1: the batch's last chunk counts as outside, so a
    // correct kernel trips the check and pbg_check must report it); 0 otherwise
    uint32_t bounds_shrink;
};

// PBG_BOUNDS debug build (make bounds -> popbam_amd/variants/bounds/libpopbam_gpu.so): every key
// load of the call kernels is checked against the contract of include/popbam_gpu.h -- keys are
// read only from the 16-byte chunks of keys[] that hold keys [block_off[0], block_off[last]) --
// and a load outside sets err bit 8 (pbg_check: PBG_E_BATCH).  The product build compiles the
// checks away.
#ifdef PBG_BOUNDS
__device__ __forceinline__ void bounds_range(const Batch &B, uint64_t lo, uint64_t n) {   // key indices [lo, lo + n)
    if (n == 0) return;
    const uint32_t nblk = (B.n_sites + kSiteBlock - 1) / kSiteBlock;
    if (lo < B.block_off[0] || lo + n + B.bounds_shrink > B.block_off[nblk]) atomicOr(B.err, 8);
}
__device__ __forceinline__ void bounds_chunk(const Batch &B, uint64_t c) {   // 16-byte chunk c of keys[]
    const uint32_t nblk = (B.n_sites + kSiteBlock - 1) / kSiteBlock;
    if (8 * c + 8 <= B.block_off[0] || 8 * c + B.bounds_shrink >= B.block_off[nblk]) atomicOr(B.err, 8);
}
#define PBG_BOUNDS_KEYS(B, lo, n) ::pbg::bounds_range((B), (lo), (n))
#define PBG_BOUNDS_CHUNK(B, c) ::pbg::bounds_chunk((B), (c))
#else
#define PBG_BOUNDS_KEYS(B, lo, n) ((void)0)
#define PBG_BOUNDS_CHUNK(B, c) ((void)0)
#endif

// Store checks of the same build: every device store and bump of the call kernels names its
// array's class and is checked against that array's allocation (DeepBufs::*_n / *_chk, the
// batch's n_sites for rows; the statistics pool against its capacity).  An index at or past
// the checked length sets the class's err bit (pbg_check reports which); an index past the real
// allocation is also not stored, so a bounds build reports a wild store instead of faulting.
// The product build compiles every guard to `true`.
constexpr int kErrQueue = 16;    // call_scan_kernel's 48-byte queue records (D.raw, the block's region)
constexpr int kErrDeep = 32;     // deep-task list entries (D.tasks)
constexpr int kErrInfo = 64;     // per-(position, sample) info bytes (D.info)
constexpr int kErrRow = 128;     // packed rows
constexpr int kErrBlock = 256;   // per-block bookkeeping: D.pend, D.blk_cnt, D.sites
constexpr int kErrWords = 512;   // consensus words (cb_out)
constexpr int kErrPool = 1024;   // statistics workspace (pool / ZnS lists)
constexpr int kErrCompact = 2048;   // (every build) a compact piece flagged a task that cannot be reference-only
#ifdef PBG_BOUNDS
__device__ __forceinline__ bool store_guard(int *err, uint64_t idx, uint64_t chk, uint64_t lim, int bit) {
    if (idx >= chk) atomicOr(err, bit);
    return idx < lim;
}
#define PBG_STORE_OK(err, idx, chk, lim, bit) \
    ::pbg::store_guard((err), (uint64_t)(idx), (uint64_t)(chk), (uint64_t)(lim), (bit))
#else
#define PBG_STORE_OK(err, idx, chk, lim, bit) true
#endif
// the classes' guards (D: DeepBufs, n_sites: the batch's positions = its rows)
#define PBG_ROW_OK(err, D, n_sites, s) PBG_STORE_OK(err, s, (n_sites) / (D).rows_div, n_sites, ::pbg::kErrRow)
#define PBG_INFO_OK(err, D, i) PBG_STORE_OK(err, i, (D).info_chk, (D).info_n, ::pbg::kErrInfo)
#define PBG_BLK_OK(err, D, b) PBG_STORE_OK(err, b, (D).blk_chk, (D).blk_n, ::pbg::kErrBlock)
#define PBG_SITES_OK(err, D, i) PBG_STORE_OK(err, i, (D).sites_chk, (D).sites_n, ::pbg::kErrBlock)
#define PBG_TASK_OK(err, D, i) PBG_STORE_OK(err, i, (D).tasks_chk, (D).tasks_n, ::pbg::kErrDeep)
#define PBG_WORD_OK(err, D, n_words, i) PBG_STORE_OK(err, i, (n_words) / (D).words_div, n_words, ::pbg::kErrWords)

// kernel launchers (defined in call_kernel.hip / stats_kernel.hip)
// n_cu: the context device's CU count (sizes the persistent queue kernel's grid).
hipError_t launch_call_sites(int row_bytes, const DevParams &P, const DevTables &T, const Batch &B, uint32_t cap,
                             void *rows, uint64_t *cb, int *err, const struct DeepBufs &D, hipStream_t stream,
                             hipEvent_t ev0, hipEvent_t ev1, int n_cu);
size_t call_sites_lds_bytes(int n, uint32_t cap);
// synthetic batch: k / rmsq / ref + per-block key totals, then an exclusive scan of the totals
// into block_off (scratch: one u64 per 1024 blocks), then the keys
hipError_t launch_synth(const DevParams &P, uint64_t seed, int contig, int mean_depth, int64_t pos0, uint32_t n_sites,
                        uint8_t *ref, void *k, uint32_t *rmsq, uint64_t *block_off, uint16_t *keys,
                        uint64_t keys_cap, uint64_t *scratch, const uint16_t *tmpl, int *err, hipStream_t stream);
// the read-template table of a seed (kTmplSize u16 entries, 16-byte aligned)
hipError_t launch_synth_tmpl(uint64_t seed, uint16_t *tmpl, hipStream_t stream);
size_t synth_scratch_words(uint32_t n_sites);
hipError_t launch_window_stats(int row_bytes, const DevParams &P, const DevTables &T, const void *rows,
                               uint32_t n_rows, uint32_t n_win, const StatsArgs &A, hipStream_t stream, int n_cu);

}  // namespace pbg
