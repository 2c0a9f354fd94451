// stats_kernel.hip -- per-window population-genetics statistics on gfx950.
//
// One workgroup (256 threads) per window.  Rows of the window are streamed once from HBM
// (coalesced, row_bytes per position); counted positions are tallied with wave ballots and
// the segregating rows are compacted, in order, into LDS (global workspace when a window has
// more than kSegCap of them).  Derived-allele bitplanes per sample are built with wave64
// ballots (one u64 word = 64 segregating sites), which turns the pairwise-difference matrix
// (calc_diff_matrix, pop_nucdiv.cpp:242-256) into popcounts of XORed words.
//
// The floating-point epilogues run in single lanes in exactly the reference's order
// (sequential double sums; x86 rounding reproduced: -ffp-contract=off, IEEE div/sqrt), so
// integer outputs and all ZnS / omega / D / H / pi values are bit-identical:
//   nucdiv   calc_nucdiv           pop_nucdiv.cpp:206-239 (+ /num_sites of print_nucdiv)
//   sfs      calc_sfs              pop_sfs.cpp:227-291
//   ld       calc_zns / calc_omegamax / calc_wall   pop_ld.cpp:201-458
//   diverge  calc_diverge + print  pop_diverge.cpp:220-257, 496-574
//   haplo    calc_nhaps / calc_ehhs / calc_minDxy    pop_haplo.cpp:208-363
#include "pbg_common.h"

namespace pbg {

namespace {

template <int RB>
__device__ __forceinline__ void load_row(const void *rows, int64_t i, uint64_t &types, bool &counted, bool &seg, int n) {
    if constexpr (RB == 16) {
        ulonglong2 v = reinterpret_cast<const ulonglong2 *>(rows)[i];
        types = v.x;
        counted = (v.y >> 62) & 1;
        seg = (v.y >> 63) & 1;
    } else {
        uint64_t v;
        if constexpr (RB == 2) v = reinterpret_cast<const uint16_t *>(rows)[i];
        else if constexpr (RB == 4) v = reinterpret_cast<const uint32_t *>(rows)[i];
        else v = reinterpret_cast<const uint64_t *>(rows)[i];
        constexpr int W = RB * 8;
        counted = (v >> (W - 2)) & 1;
        seg = (v >> (W - 1)) & 1;
        types = v & ((W == 64) ? 0x3FFFFFFFFFFFFFFFULL : ((1ULL << (W - 2)) - 1));
    }
}

__device__ __forceinline__ unsigned pc(uint64_t x) { return (unsigned)__popcll(x); }

// x86 SSE produces the "default NaN" (sign bit set) for invalid operations; glibc prints it
// as "-nan".  Canonicalise device NaNs the same way before they reach the formatter.
__device__ __forceinline__ double x86nan(double v) { return (v != v) ? __longlong_as_double(0xFFF8000000000000LL) : v; }

// r^2 of pop_ld.cpp:239-243 from the host table (same expression, same rounding)
__device__ __forceinline__ double r2lookup(const DevTables &T, int p, int np1, unsigned m1, unsigned m2, unsigned c11) {
    return T.r2[T.r2_off[p] + ((int)m1 * np1 + (int)m2) * np1 + (int)c11];
}

}  // namespace

template <int RB>
__global__ __launch_bounds__(kBlockThreads) void window_stats_kernel(DevParams P, DevTables T, const void *__restrict__ rows,
                                                                     uint32_t n_rows, uint32_t n_win, StatsArgs A) {
    __shared__ uint64_t s_seg[kSegCap];
    __shared__ uint64_t s_plane[kPlaneCap];
    __shared__ uint16_t s_diff[PBG_MAX_SAMPLES * PBG_MAX_SAMPLES];
    __shared__ uint32_t s_wcnt[kBlockThreads / 64][2];
    __shared__ int32_t s_scratch[PBG_MAX_POPS * (PBG_MAX_SAMPLES + 2)];
    __shared__ int32_t s_ns, s_S;

    const uint32_t w = blockIdx.x;
    if (w >= n_win) return;
    const int n = P.n, np = P.npops;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t wb = A.wins[w].beg, we = A.wins[w].end;
    const int64_t len = we > wb ? we - wb : 0;

    // ---- pass 1: counted / segregating totals
    uint32_t my_c = 0, my_s = 0;
    for (int64_t i = tid; i < len; i += kBlockThreads) {
        uint64_t t;
        bool c, s;
        load_row<RB>(rows, wb + i, t, c, s, n);
        my_c += c;
        my_s += s;
    }
    for (int o = 32; o > 0; o >>= 1) {
        my_c += __shfl_down(my_c, o, 64);
        my_s += __shfl_down(my_s, o, 64);
    }
    if (lane == 0) { s_wcnt[wv][0] = my_c; s_wcnt[wv][1] = my_s; }
    __syncthreads();
    if (tid == 0) {
        int a = 0, b = 0;
        for (int k = 0; k < kBlockThreads / 64; ++k) { a += (int)s_wcnt[k][0]; b += (int)s_wcnt[k][1]; }
        s_ns = a;
        s_S = b;
    }
    __syncthreads();
    const int num_sites = s_ns, S = s_S;
    const bool ld_next = (A.stats & (PBG_S_ZNS | PBG_S_OMEGA | PBG_S_WALL)) != 0;
    uint64_t *seg = (S <= kSegCap && !ld_next) ? s_seg : (A.ws + A.ws_off[w]);

    // ---- pass 2: ordered compaction of segregating rows (ballot + cross-wave prefix)
    {
        int base = 0;
        for (int64_t c0 = 0; c0 < len; c0 += kBlockThreads) {
            int64_t i = c0 + tid;
            uint64_t t = 0;
            bool c = false, s = false;
            if (i < len) load_row<RB>(rows, wb + i, t, c, s, n);
            uint64_t m = __ballot(s);
            int before = (int)__popcll(m & ((1ULL << lane) - 1));
            __syncthreads();
            if (lane == 0) s_wcnt[wv][0] = (uint32_t)__popcll(m);
            __syncthreads();
            int wofs = 0, tot = 0;
            for (int k = 0; k < kBlockThreads / 64; ++k) {
                if (k < wv) wofs += (int)s_wcnt[k][0];
                tot += (int)s_wcnt[k][0];
            }
            if (s) seg[base + wofs + before] = t;
            base += tot;
        }
    }
    __syncthreads();

    // types of the j-th segregating site: seg[j] (== types[hap.idx[j]] in the reference)
    const int nwords = S > 0 ? (S + 63) / 64 : 1;
    const bool need_planes = (A.stats & (PBG_S_NUCDIV | PBG_S_DIV_IND | PBG_S_HAP_K | PBG_S_HAP_EHHS | PBG_S_HAP_DXY |
                                         PBG_S_TREE)) != 0;
    uint64_t *plane = nullptr;
    if (need_planes) {
        plane = (n * nwords <= kPlaneCap) ? s_plane : (A.ws + A.ws_off[w] + ws_plane_off(len));
        // plane[v*nwords + k] bit b = sample v derived at segregating site 64k+b (hap.seq)
        for (int k = wv; k < nwords; k += kBlockThreads / 64) {
            int j = k * 64 + lane;
            uint64_t t = j < S ? seg[j] : 0;
            for (int v = 0; v < n; ++v) {
                uint64_t m = __ballot((t >> v) & 1);
                if (lane == 0) plane[v * nwords + k] = m;
            }
        }
        __syncthreads();
        // calc_diff_matrix: u16 accumulation (wraps, Appendix A.7)
        const int npair = n * n;
        for (int pr = tid; pr < npair; pr += kBlockThreads) {
            int v = pr / n, u = pr - v * n;
            uint32_t d = 0;
            if (v != u)
                for (int k = 0; k < nwords; ++k) d += pc(plane[v * nwords + k] ^ plane[u * nwords + k]);
            s_diff[pr] = (uint16_t)(d & 0xFFFF);
        }
        __syncthreads();
    }

    const pbg_window_out &O = A.out;
    if (tid == 0) {
        if (O.num_sites) O.num_sites[w] = num_sites;
        if (O.segsites) O.segsites[w] = S;
    }
    const int npairs = np * (np - 1);

    // ---- nucdiv (one lane): integer sums are exact in double, as in the reference
    if ((A.stats & PBG_S_NUCDIV) && tid == 0) {
        for (int i = 0; i < np; i++)
            for (int j = i; j < np; j++) {
                double acc = 0.0;
                for (int v = 0; v < n - 1; v++)
                    for (int u = v + 1; u < n; u++)
                        if (((P.pop_mask[i] >> v) & 1) && ((P.pop_mask[j] >> u) & 1)) acc += (double)s_diff[v * n + u];
                if (i != j) {
                    acc *= 1.0 / (double)(P.pop_n[i] * P.pop_n[j]);
                    if (O.dxy) O.dxy[(size_t)w * npairs + i * np + (j - (i + 1))] = x86nan(acc / num_sites);
                } else {
                    acc *= 2.0 / (double)(P.pop_n[i] * (P.pop_n[i] - 1));
                    if (acc != acc) acc = 0.0;
                    if (O.pi) O.pi[(size_t)w * np + i] = x86nan(acc / num_sites);
                }
            }
    }

    // ---- sfs (lane per population)
    if ((A.stats & PBG_S_SFS) && tid >= 64 && tid < 64 + np) {
        const int i = tid - 64;
        const int nn = P.pop_n[i];
        int *sfs = s_scratch + i * (PBG_MAX_SAMPLES + 2);
        for (int j = 0; j <= nn; ++j) sfs[j] = 0;
        int S_i = 0;
        for (int j = 0; j < S; j++) {
            uint64_t t = seg[j];
            uint64_t pt = t & P.pop_mask[i];
            unsigned freq;
            if ((P.flag & PBG_F_OUTGROUP) && ((t >> A.outidx) & 1)) freq = (unsigned)(uint16_t)(nn - (int)pc(pt));
            else freq = pc(pt);
            ++sfs[freq];
            if (freq > 0 && (int)freq < nn) ++S_i;
        }
        double td = 0.0, fwh = 0.0;
        if (S_i > 0 && nn > 1) {
            const double a1 = T.a1[nn], a2 = T.a2[nn], e1 = T.e1[nn], e2 = T.e2[nn], a2n1 = T.a2[nn + 1];
            for (int j = 1; j < nn; j++) {
                td += sfs[j] * (((2.0 * j * (nn - j)) / (nn * (nn - 1))) - (1.0 / a1));
                fwh += sfs[j] * ((1.0 / a1) - ((double)j / (nn - 1)));
            }
            td /= sqrt(e1 * S_i + e2 * S_i * (S_i - 1));
            fwh /= sqrt(((nn - 2) * (S_i / a1) / (6.0 * (nn - 1))) +
                                  ((S_i * (S_i - 1) / ((a1 * a1) + a2)) *
                                   (18.0 * (nn * nn) * (3.0 * nn + 2.0) * a2n1 - (88.0 * nn * nn * nn + 9.0 * (nn * nn) - 13.0 * nn + 6.0)) /
                                   (9.0 * nn * ((nn - 1) * (nn - 1)))));
        } else {
            td = __longlong_as_double(0x7FF8000000000000LL);
            fwh = td;
        }
        if (O.td) O.td[(size_t)w * np + i] = td;
        if (O.fwh) O.fwh[(size_t)w * np + i] = fwh;
    }

    // ZnS / omega_max / Wall's B,Q are serial chains per (window, population): they run in
    // window_ld_kernel, one lane per chain, over the segregating lists left in the workspace.
    if (tid == 0 && A.seg_count) A.seg_count[w] = S;

    // ---- ld -o 0 (ZnS, pop_ld.cpp:201-252): per population, the ordered list of segregating
    // rows variable within it (masked to the population) for window_zns_kernel, and num_snps
    // (variable sites among the first S-1, plus the final unconditional increment)
    if ((A.stats & PBG_S_ZNS) && A.var_count) {
        __shared__ int32_t s_lastvar;
        for (int i = 0; i < np; ++i) {
            const uint64_t pm = P.pop_mask[i];
            const int nn = P.pop_n[i], mf = A.min_freq;
            uint64_t *vl = A.ws + A.ws_off[w] + ws_list_off(len, n) + (uint64_t)i * (uint64_t)(len + 1);
            int base = 0;
            for (int c0 = 0; c0 < S; c0 += kBlockThreads) {
                const int j = c0 + tid;
                uint64_t t = 0;
                bool v = false;
                if (j < S) {
                    t = seg[j] & pm;
                    const int m = (int)pc(t);
                    v = m >= mf && m <= nn - mf;
                    if (j == S - 1) s_lastvar = v ? 1 : 0;
                }
                const uint64_t bm = __ballot(v);
                const int before = (int)__popcll(bm & ((1ULL << lane) - 1));
                __syncthreads();
                if (lane == 0) s_wcnt[wv][0] = (uint32_t)__popcll(bm);
                __syncthreads();
                int wofs = 0, tot = 0;
                for (int k = 0; k < kBlockThreads / 64; ++k) {
                    if (k < wv) wofs += (int)s_wcnt[k][0];
                    tot += (int)s_wcnt[k][0];
                }
                if (v) vl[base + wofs + before] = t;
                base += tot;
            }
            __syncthreads();
            if (tid == 0) {
                const int ns = S >= 1 ? base - s_lastvar + 1 : 0;
                A.var_count[(size_t)w * np + i] = base;
                A.ld_ns[(size_t)w * np + i] = ns;
                if (A.out.ld_snps) A.out.ld_snps[(size_t)w * np + i] = ns;
            }
        }
    }

    // ---- diverge -o 0 (lane per sample): u16 accumulation of derived counts
    if ((A.stats & PBG_S_DIV_IND) && tid < n) {
        uint32_t d = 0;
        for (int k = 0; k < nwords; ++k) d += pc(plane[tid * nwords + k]);
        double pd = (double)(d & 0xFFFF) / num_sites;
        double v = A.jc ? -0.75 * log(1.0 - pd * (4.0 / 3.0)) : pd;
        if (O.div_ind) O.div_ind[(size_t)w * n + tid] = x86nan(v);
    }
    // ---- tree: treeData's diff_matrix (calc_diff_matrix, pop_tree.cpp:472-494), u16 values;
    //      taxon 0 is the reference (row = the sample's derived count), taxon i+1 sample i
    if ((A.stats & PBG_S_TREE) && O.tree_diff) {
        const int nt = n + 1;
        int32_t *td = O.tree_diff + (size_t)w * nt * nt;
        for (int pr = tid; pr < nt * nt; pr += kBlockThreads) {
            const int a = pr / nt, b = pr - a * nt;
            int32_t v = 0;
            if (a != b && (a == 0 || b == 0)) {
                const int sm = a + b - 1;
                uint32_t d = 0;
                for (int k = 0; k < nwords; ++k) d += pc(plane[sm * nwords + k]);
                v = (int32_t)(d & 0xFFFF);
            } else if (a != b) {
                v = s_diff[(a - 1) * n + (b - 1)];
            }
            td[pr] = v;
        }
    }
    // ---- diverge -o 1 (lane per population)
    if ((A.stats & PBG_S_DIV_POP) && tid >= 64 && tid < 64 + np) {
        const int i = tid - 64, nn = P.pop_n[i];
        int segs = 0;
        uint32_t fixed = 0;
        for (int j = 0; j < S; j++) {
            uint64_t t = seg[j];
            uint64_t pt = t & P.pop_mask[i];
            unsigned freq;
            if ((P.flag & PBG_F_OUTGROUP) && ((t >> A.outidx) & 1)) freq = (unsigned)(uint16_t)(nn - (int)pc(pt));
            else freq = pc(pt);
            if (freq > 0 && (int)freq < nn) ++segs;
            else if ((int)freq == nn) ++fixed;
        }
        fixed &= 0xFFFF;
        double pd = (P.flag & PBG_F_SUBSTITUTE) ? (double)fixed / num_sites : (double)(fixed + segs) / num_sites;
        double v = A.jc ? -0.75 * log(1.0 - pd * (4.0 / 3.0)) : pd;
        if (O.div_fixed) O.div_fixed[(size_t)w * np + i] = (int32_t)fixed;
        if (O.div_seg) O.div_seg[(size_t)w * np + i] = segs;
        if (O.div_pop) O.div_pop[(size_t)w * np + i] = x86nan(v);
    }

    // ---- haplo K / Kdiv and EHHS (lane per population)
    if ((A.stats & (PBG_S_HAP_K | PBG_S_HAP_EHHS)) && tid >= 64 && tid < 64 + np) {
        const int i = tid - 64, nelem = P.pop_n[i];
        int nh = 0;
        double hdiv;
        int *b = s_scratch + i * (PBG_MAX_SAMPLES + 2);
        if (nelem > 1) {
            int c = 0;
            for (int j = 0; j < n; j++)
                if ((P.pop_mask[i] >> j) & 1) b[c++] = j;
            // local indices j,k index the global diff matrix (A.11)
            for (int j = 0; j < nelem - 1; j++)
                for (int k = j + 1; k < nelem; k++)
                    if (s_diff[j * n + k] == 0 && b[k] > b[j]) b[k] = j;
            int ff = 0;
            for (int j = 0; j < nelem; j++) {
                int f = 0;
                for (int q = 0; q < nelem; q++) f += b[q] == j;
                if (f > 0) ++nh;
                ff += f * f;
            }
            double sh = (double)(ff) / (double)(nelem * nelem);
            hdiv = 1.0 - ((1.0 - sh) * (double)(nelem / (nelem - 1)));
        } else {
            nh = 1;
            hdiv = 1.0;
        }
        if (A.stats & PBG_S_HAP_K) {
            if (O.nhaps) O.nhaps[(size_t)w * np + i] = nh;
            if (O.hap_val) O.hap_val[(size_t)w * np + i] = x86nan(1.0 - hdiv);
        } else {
            double e;
            if (nelem < 4) {
                e = __longlong_as_double(0x7FF8000000000000LL);
            } else {
                // max multiplicity among non-singleton partitions, ties -> smallest value
                // (std::list sort + unique + remove, pop_haplo.cpp:273-313)
                const uint64_t pm = P.pop_mask[i];
                int best = 0;
                uint64_t max_site = 0;
                for (int j = 0; j < S; j++) {
                    uint64_t pt = seg[j] & pm;
                    unsigned f = pc(pt);
                    if (!(f > 1 && (int)f < nelem - 1)) continue;
                    int cnt = 0;
                    for (int q = 0; q < S; q++) cnt += (seg[q] & pm) == pt;
                    int part_count = cnt + 1;
                    if (part_count > best || (part_count == best && pt < max_site)) {
                        best = part_count;
                        max_site = pt;
                    }
                }
                unsigned popf = pc(max_site);
                int pn = nelem;
                double sh = (1.0 - ((double)((int)(popf * popf) + ((pn - (int)popf) * (pn - (int)popf))) / (pn * pn))) *
                            (double)(pn / (pn - 1));
                e = hdiv / (1.0 - sh);
            }
            if (O.hap_val) O.hap_val[(size_t)w * np + i] = e;
        }
    }

    // ---- haplo -o 2: pi (not divided by num_sites), dxy and min pairwise differences
    if ((A.stats & PBG_S_HAP_DXY) && tid == 0) {
        for (int i = 0; i < np; i++)
            for (int j = i; j < np; j++) {
                double acc = 0.0;
                int mn = 65535;   // UINT_MAX narrowed to u16 (A.7)
                for (int v = 0; v < n - 1; v++)
                    for (int u = v + 1; u < n; u++)
                        if (((P.pop_mask[i] >> v) & 1) && ((P.pop_mask[j] >> u) & 1)) {
                            acc += (double)s_diff[v * n + u];
                            if (i != j) mn = mn < (int)s_diff[v * n + u] ? mn : (int)s_diff[v * n + u];
                        }
                if (i != j) {
                    acc *= 1.0 / (double)(P.pop_n[i] * P.pop_n[j]);
                    int pi = i * np + (j - (i + 1));
                    if (O.hap_dxy) O.hap_dxy[(size_t)w * npairs + pi] = x86nan(acc);
                    if (O.hap_min) O.hap_min[(size_t)w * npairs + pi] = mn;
                } else {
                    acc *= 2.0 / (double)(P.pop_n[i] * (P.pop_n[i] - 1));
                    if (acc != acc) acc = 0.0;
                    if (O.hap_val) O.hap_val[(size_t)w * np + i] = acc;
                }
            }
    }
}


// ZnS (calc_zns, pop_ld.cpp:201-252): per (window, population) chain, the sum of r^2 over
// all pairs a < b of its variable sites in the reference's order (a ascending, then b), as
// one dependent double add per pair.  A wave owns kZnsChains chains: all 64 lanes compute the
// next 64 r^2 values of one row of one chain at a time (popcounts + r^2 table lookups),
// writing them to LDS; then lane j adds chain j's values in order.  The parallel part is
// spread over the wave, the serial part runs kZnsChains chains side by side.
#ifndef PBG_ZNS_CHAINS
#define PBG_ZNS_CHAINS 8
#endif
constexpr int kZnsChains = PBG_ZNS_CHAINS;
constexpr int kZnsCap = 256;   // variable sites per chain staged in LDS (larger: read from HBM)

__global__ __launch_bounds__(64) void window_zns_kernel(DevParams P, DevTables T, uint32_t n_win, StatsArgs A,
                                                        int r2_lds) {
    extern __shared__ double s_r2[];
    __shared__ uint64_t s_t[kZnsChains][kZnsCap];
    __shared__ double s_buf[kZnsChains][72];   // 64 values + zero tail for the groups of 8
    const int lane = threadIdx.x, np = P.npops;
    const uint32_t nch = n_win * (uint32_t)np;
    const uint32_t c0 = blockIdx.x * kZnsChains;
    for (int i = lane; i < r2_lds; i += 64) s_r2[i] = T.r2[i];
    s_buf[lane >> 3][64 + (lane & 7)] = 0.0;

    int Vc[kZnsChains], np1c[kZnsChains], offc[kZnsChains];
    const uint64_t *Lg[kZnsChains];
    int Vmax = 0;
#pragma unroll
    for (int j = 0; j < kZnsChains; ++j) {
        const uint32_t ch = c0 + j;
        Vc[j] = 0;
        np1c[j] = 1;
        offc[j] = 0;
        Lg[j] = A.ws;
        if (ch < nch) {
            const uint32_t w = ch / (uint32_t)np;
            const int i = (int)(ch - w * (uint32_t)np);
            const int64_t len = A.wins[w].end > A.wins[w].beg ? A.wins[w].end - A.wins[w].beg : 0;
            Vc[j] = A.var_count[ch];
            np1c[j] = P.pop_n[i] + 1;
            offc[j] = T.r2_off[i];
            Lg[j] = A.ws + A.ws_off[w] + ws_list_off(len, P.n) + (uint64_t)i * (uint64_t)(len + 1);
        }
        Vmax = Vc[j] > Vmax ? Vc[j] : Vmax;
    }
    const bool fast = Vmax <= kZnsCap && r2_lds > 0;   // workgroup-uniform
    if (fast) {
#pragma unroll
        for (int j = 0; j < kZnsChains; ++j)
            for (int b = lane; b < Vc[j]; b += 64) s_t[j][b] = Lg[j][b];
    }
    __syncthreads();
    // s_buf rows are zero-padded: adding +0.0 leaves a sum of r^2 values (>= +0) bit-unchanged,
    // so each segment is summed in fixed groups of 8 whatever the chains' row lengths
    double acc = 0.0;
    for (int a = 0; a < Vmax - 1; ++a) {
        for (int b0 = 0; b0 < Vmax - 1 - a; b0 += 64) {
            if (fast) {   // straight-line over the chains: loads of all chains in flight together
                uint64_t ta[kZnsChains], tb[kZnsChains];
                bool ok[kZnsChains];
#pragma unroll
                for (int j = 0; j < kZnsChains; ++j) {
                    const int L = Vc[j] - 1 - a;
                    ok[j] = b0 + lane < L;
                    const int ac = L > 0 ? a : 0, bc = ok[j] ? a + 1 + b0 + lane : 0;
                    ta[j] = s_t[j][ac];
                    tb[j] = s_t[j][bc];
                    ta[j] = L > 0 ? ta[j] : 0;
                    tb[j] = ok[j] ? tb[j] : 0;
                }
                double v[kZnsChains];
#pragma unroll
                for (int j = 0; j < kZnsChains; ++j) {
                    const int np1 = np1c[j];
                    v[j] = s_r2[offc[j] + ((int)pc(ta[j]) * np1 + (int)pc(tb[j])) * np1 + (int)pc(ta[j] & tb[j])];
                }
#pragma unroll
                for (int j = 0; j < kZnsChains; ++j) s_buf[j][lane] = ok[j] ? v[j] : 0.0;
            } else {      // a chain above kZnsCap, or r^2 tables too large for LDS: from HBM
                for (int j = 0; j < kZnsChains; ++j) {
                    const int L = Vc[j] - 1 - a;
                    double v = 0.0;
                    if (b0 + lane < L) {
                        const uint64_t ta = Lg[j][a], tb = Lg[j][a + 1 + b0 + lane];
                        const int np1 = np1c[j];
                        v = T.r2[offc[j] + ((int)pc(ta) * np1 + (int)pc(tb)) * np1 + (int)pc(ta & tb)];
                    }
                    s_buf[j][lane] = v;
                }
            }
            __syncthreads();
            const int seg = min(64, Vmax - 1 - a - b0);   // longest segment of the wave's chains
            if (lane < kZnsChains) {
                for (int l = 0; l < seg; l += 8) {
                    double x[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = s_buf[lane][l + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) acc += x[u];
                }
            }
            __syncthreads();
        }
    }
    if (lane < kZnsChains && c0 + lane < nch) {
        const uint32_t ch = c0 + lane;
        const uint32_t w = ch / (uint32_t)np;
        double val = 0.0;
        if (A.seg_count[w] >= 1) {
            const int ns = A.ld_ns[ch];
            val = acc * (2.0 / (ns * (ns - 1)));
        }
        if (A.out.ld_val) A.out.ld_val[ch] = x86nan(val);
    }
}

// Serial LD chains, one lane per chain (pop_ld.cpp:201-458), reading the ordered segregating
// lists window_stats_kernel compacted into the workspace.  Lanes of a wave belong to
// different windows, so the dependent double additions of 64 chains overlap.
__global__ __launch_bounds__(kBlockThreads) void window_ld_kernel(DevParams P, DevTables T, uint32_t n_win, StatsArgs A) {
    __shared__ double s_r2[4096];
    const int n = P.n, np = P.npops;
    int r2_total = 0;
    for (int i = 0; i < np; ++i) r2_total += (P.pop_n[i] + 1) * (P.pop_n[i] + 1) * (P.pop_n[i] + 1);
    const bool r2_lds = r2_total <= 4096;
    if (r2_lds)
        for (int i = threadIdx.x; i < r2_total; i += kBlockThreads) s_r2[i] = T.r2[i];
    __syncthreads();
    const double *r2tab = r2_lds ? s_r2 : T.r2;
    const pbg_window_out &O = A.out;
    const uint32_t gid = blockIdx.x * kBlockThreads + threadIdx.x;
    if (A.stats & PBG_S_WALL) {
        // one chain per window: last_type is shared by all populations (Appendix A.9)
        const uint32_t w = gid;
        if (w >= n_win) return;
        const int64_t len = A.wins[w].end > A.wins[w].beg ? A.wins[w].end - A.wins[w].beg : 0;
        const int S = A.seg_count[w];
        const uint64_t *seg = A.ws + A.ws_off[w];
        int ns[PBG_MAX_POPS], cong[PBG_MAX_POPS], part[PBG_MAX_POPS], nu[PBG_MAX_POPS];
        for (int j = 0; j < np; j++) ns[j] = cong[j] = part[j] = nu[j] = 0;
        uint64_t *uniq = A.ws + A.ws_off[w] + ws_list_off(len, n);   // np slices of (len+1)
        uint64_t last_type = 0;
        for (int i = 0; i < S; i++) {
            const uint64_t t = seg[i];
            for (int j = 0; j < np; j++) {
                const uint64_t type = t & P.pop_mask[j];
                const uint64_t comp = ~t & P.pop_mask[j];
                uint64_t *u = uniq + (uint64_t)j * (uint64_t)(len + 1);
                if (type > 0 && type < P.pop_mask[j]) {
                    if (ns[j] == 0) {
                        u[nu[j]++] = type;
                        last_type = type;
                        ns[j]++;
                    } else {
                        if (type == last_type || comp == last_type) {
                            cong[j]++;
                            bool seen = false;
                            for (int q = 0; q < nu[j]; q++) seen |= (u[q] == type) || (u[q] == comp);
                            if (!seen) {
                                u[nu[j]++] = type;
                                part[j]++;
                            }
                        }
                        ns[j]++;
                        last_type = type;
                    }
                }
            }
        }
        for (int j = 0; j < np; j++) {
            double b = 0.0, q = 0.0;
            if (S >= 1) {
                b = (double)cong[j] / (double)(ns[j] - 1);
                q = (double)(cong[j] + part[j]) / ns[j];
            }
            if (O.ld_snps) O.ld_snps[(size_t)w * np + j] = ns[j];
            if (O.ld_val) O.ld_val[(size_t)w * np + j] = x86nan(b);
            if (O.ld_q) O.ld_q[(size_t)w * np + j] = x86nan(q);
        }
        return;
    }
    if (gid >= n_win * (uint32_t)np) return;
    const uint32_t w = gid / np;
    const int i = (int)(gid - w * np);
    const int64_t len = A.wins[w].end > A.wins[w].beg ? A.wins[w].end - A.wins[w].beg : 0;
    const int S = A.seg_count[w];
    const uint64_t *seg = A.ws + A.ws_off[w];
    const int nn = P.pop_n[i], np1 = nn + 1, mf = A.min_freq;
    const uint64_t pm = P.pop_mask[i];
    const double *r2p = r2tab + T.r2_off[i];
    auto variable = [&](unsigned m) { return (int)m >= mf && (int)m <= nn - mf; };
    int ns = 0;
    double val = 0.0;
    {   // calc_omegamax pop_ld.cpp:254-373 (ZnS runs in window_zns_kernel) (sums accumulate across partitions, A.8)
        if (S >= 1) {
            int V = 0;
            uint64_t *vt = A.ws + A.ws_off[w] + ws_list_off(len, n) + (uint64_t)i * (uint64_t)(len + 1);
            for (int j = 0; j < S; j++) {
                const uint64_t t = seg[j] & pm;
                if (variable(pc(t))) {
                    if (j < S - 1) ++ns;
                    vt[V++] = t;
                }
            }
            ++ns;
            auto r2 = [&](int a, int b) -> double {   // a < b; 0 beyond the variable sites
                if (b >= V) return 0.0;
                const uint64_t ta = vt[a], tb = vt[b];
                return r2p[((int)pc(ta) * np1 + (int)pc(tb)) * np1 + (int)pc(ta & tb)];
            };
            double sl = 0, sr = 0, sb = 0;
            for (int ii = 1; ii < ns - 1; ii++) {
                for (int k = 0; k < ii; k++)
                    for (int m = k + 1; m <= ii; m++) sl += r2(k, m);
                for (int k = ii + 1; k < ns; k++)
                    for (int m = 0; m <= ii; m++) sb += r2(m, k);
                for (int k = ii + 1; k < ns - 1; k++)
                    for (int m = k + 1; m < ns; m++) sr += r2(k, m);
                const int left = ii + 1, right = ns - left;
                double omega = (sl + sr) / (((left * (left - 1)) / 2.0) + ((right * (right - 1)) / 2.0));
                omega *= left * right / sb;
                val = omega > val ? omega : val;
            }
        }
    }
    if (O.ld_snps) O.ld_snps[(size_t)w * np + i] = ns;
    if (O.ld_val) O.ld_val[(size_t)w * np + i] = x86nan(val);
}

template __global__ void window_stats_kernel<2>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<4>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<8>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<16>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);

}  // namespace pbg

namespace pbg {

hipError_t launch_window_stats(int rb, const DevParams &P, const DevTables &T, const void *rows, uint32_t n_rows,
                               uint32_t n_win, const StatsArgs &A, hipStream_t stream) {
    if (n_win == 0) return hipSuccess;
    dim3 g(n_win), b(kBlockThreads);
    switch (rb) {
        case 2: hipLaunchKernelGGL(window_stats_kernel<2>, g, b, 0, stream, P, T, rows, n_rows, n_win, A); break;
        case 4: hipLaunchKernelGGL(window_stats_kernel<4>, g, b, 0, stream, P, T, rows, n_rows, n_win, A); break;
        case 8: hipLaunchKernelGGL(window_stats_kernel<8>, g, b, 0, stream, P, T, rows, n_rows, n_win, A); break;
        default: hipLaunchKernelGGL(window_stats_kernel<16>, g, b, 0, stream, P, T, rows, n_rows, n_win, A); break;
    }
    const uint32_t ld = A.stats & (PBG_S_ZNS | PBG_S_OMEGA | PBG_S_WALL);
    if (ld) {
        if (ld != PBG_S_ZNS && ld != PBG_S_OMEGA && ld != PBG_S_WALL) return hipErrorInvalidValue;
        const uint32_t chains = (ld == PBG_S_WALL) ? n_win : n_win * (uint32_t)P.npops;
        if (ld == PBG_S_ZNS) {
            int r2_total = 0;
            for (int i = 0; i < P.npops; ++i) r2_total += (P.pop_n[i] + 1) * (P.pop_n[i] + 1) * (P.pop_n[i] + 1);
            const int r2_lds = r2_total <= 4096 ? r2_total : 0;
            hipLaunchKernelGGL(window_zns_kernel, dim3((chains + kZnsChains - 1) / kZnsChains), dim3(64),
                               (size_t)r2_lds * sizeof(double), stream, P, T, n_win, A, r2_lds);
        } else {
            hipLaunchKernelGGL(window_ld_kernel, dim3((chains + kBlockThreads - 1) / kBlockThreads), b, 0, stream, P,
                               T, n_win, A);
        }
    }
    return hipGetLastError();
}

}  // namespace pbg
