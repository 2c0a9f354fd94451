// stats_kernel.hip -- per-window population-genetics statistics on gfx950.
//
// One wave (a 64-thread workgroup) per window.  The window's rows are streamed once from HBM
// with 16-byte loads (8 / 4 / 2 / 1 rows per lane per load for 2 / 4 / 8 / 16-byte rows);
// counted rows are tallied per lane and the segregating rows are compacted, in order, with a
// wave prefix sum into LDS (the window's workspace slice beyond kSegCap of them).  Derived-
// allele bitplanes per sample are built with wave64 ballots (one u64 word = 64 segregating
// sites = one hap.seq word), which turns calc_diff_matrix (pop_nucdiv.cpp:242-256) into
// popcounts of XORed words.  Every integer reduction (pairwise-difference sums per population
// pair, SFS bins, fixed / segregating counts) runs across lanes with LDS atomics: the
// reference accumulates them in double, where integer sums are exact, so order is irrelevant.
//
// The floating-point chains run in single lanes in exactly the reference's order (sequential
// double sums; x86 rounding reproduced: -ffp-contract=off, IEEE div/sqrt), so integer outputs
// and all ZnS / omega / D / H / pi values are bit-identical:
//   nucdiv   calc_nucdiv           pop_nucdiv.cpp:206-239 (+ /num_sites of print_nucdiv)
//   sfs      calc_sfs              pop_sfs.cpp:227-291   (+ the SFS bins and theta_W it implies)
//   ld       calc_zns              pop_ld.cpp:201-252    (here)
//            calc_omegamax / calc_wall   pop_ld.cpp:254-458 (window_ld_kernel, lane per chain)
//   diverge  calc_diverge + print  pop_diverge.cpp:220-257, 496-574
//   haplo    calc_nhaps / calc_ehhs / calc_minDxy    pop_haplo.cpp:208-363
//   tree     calc_diff_matrix      pop_tree.cpp:472-494
#include "pbg_common.h"

namespace pbg {
extern const int kBuildKind_stats = PBG_BUILD_KIND;   // pbg_build_info()
}

namespace pbg {

namespace {

__device__ __forceinline__ unsigned pc(uint64_t x) { return (unsigned)__popcll(x); }

// The sample bits of a row: one u64 for 2 / 4 / 8-byte rows, two for 16-byte rows (n <= 126;
// the reference's masks are one u64, n <= 64, popbam.cpp:168).  Every statistic below is
// written once over the mask type M: a bitwise and / complement, equality, the unsigned order
// (std::list::sort in calc_ehhs), popcount and a bit test.
struct M2 {
    uint64_t lo, hi;
};
__device__ __forceinline__ M2 operator&(M2 a, M2 b) { return {a.lo & b.lo, a.hi & b.hi}; }
__device__ __forceinline__ M2 operator~(M2 a) { return {~a.lo, ~a.hi}; }
__device__ __forceinline__ bool operator==(M2 a, M2 b) { return a.lo == b.lo && a.hi == b.hi; }
__device__ __forceinline__ bool operator<(M2 a, M2 b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
__device__ __forceinline__ unsigned pc(M2 x) { return pc(x.lo) + pc(x.hi); }
__device__ __forceinline__ bool nonzero(uint64_t x) { return x != 0; }
__device__ __forceinline__ bool nonzero(M2 x) { return (x.lo | x.hi) != 0; }
__device__ __forceinline__ uint32_t bit(uint64_t x, int v) { return (uint32_t)(x >> v) & 1u; }
__device__ __forceinline__ uint32_t bit(M2 x, int v) { return (uint32_t)(v < 64 ? x.lo >> v : x.hi >> (v - 64)) & 1u; }
template <class M>
__device__ __forceinline__ M pop_mask(const DevParams &P, int i);
template <>
__device__ __forceinline__ uint64_t pop_mask<uint64_t>(const DevParams &P, int i) { return P.pop_mask[i]; }
template <>
__device__ __forceinline__ M2 pop_mask<M2>(const DevParams &P, int i) { return {P.pop_mask[i], P.pop_mask_hi[i]}; }
__device__ __forceinline__ uint64_t shfl_xor_mask(uint64_t x, int o) {
    return ((uint64_t)(uint32_t)__shfl_xor((int)(x >> 32), o, 64) << 32) | (uint32_t)__shfl_xor((int)x, o, 64);
}
__device__ __forceinline__ M2 shfl_xor_mask(M2 x, int o) { return {shfl_xor_mask(x.lo, o), shfl_xor_mask(x.hi, o)}; }
template <int RB>
struct RowMask { using T = uint64_t; };
template <>
struct RowMask<16> { using T = M2; };

// x86 SSE produces the "default NaN" (sign bit set) for invalid operations; glibc prints it
// as "-nan".  Canonicalise device NaNs the same way before they reach the formatter.
__device__ __forceinline__ double x86nan(double v) { return (v != v) ? __longlong_as_double(0xFFF8000000000000LL) : v; }

// exclusive wave prefix of a lane count (DPP inclusive scan, see call_kernel.hip)
__device__ __forceinline__ uint32_t wave_incl_scan_s(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    return (uint32_t)x;
}
__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

// Row r (0 .. 16/RB - 1) of a 16-byte word of RB-byte rows (include/popbam_gpu.h row format).
template <int RB>
__device__ __forceinline__ void row_in_word(const uint4 &q, int r, typename RowMask<RB>::T &types, bool &counted,
                                            bool &seg) {
    if constexpr (RB == 16) {
        types.lo = (uint64_t)q.x | ((uint64_t)q.y << 32);
        types.hi = ((uint64_t)q.z | ((uint64_t)q.w << 32)) & 0x3FFFFFFFFFFFFFFFULL;
        counted = (q.w >> 30) & 1u;
        seg = (q.w >> 31) & 1u;
    } else {
        const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
        constexpr int W = RB * 8;
        uint64_t v;
        if constexpr (RB == 8) v = (uint64_t)wd[2 * r] | ((uint64_t)wd[2 * r + 1] << 32);
        else if constexpr (RB == 4) v = wd[r];
        else v = (wd[r >> 1] >> (16 * (r & 1))) & 0xFFFFu;
        counted = (v >> (W - 2)) & 1;
        seg = (v >> (W - 1)) & 1;
        types = v & ((W == 64) ? 0x3FFFFFFFFFFFFFFFULL : ((1ULL << (W - 2)) - 1));
    }
}

}  // namespace

WinLds stats_lds_layout(int n, int np, int sfs_stride, uint32_t stats, int r2_total, int mask_words, int segcap) {
    WinLds L{};
    uint32_t b = 0;
    auto take = [&](uint32_t bytes) {
        const uint32_t o = b;
        b += (bytes + 15) & ~15u;
        return o;
    };
    const bool planes = stats & (PBG_S_NUCDIV | PBG_S_DIV_IND | PBG_S_HAP_K | PBG_S_HAP_EHHS | PBG_S_HAP_DXY | PBG_S_TREE);
    // calc_nhaps only asks whether two samples differ: one bit per pair
    const bool zero = stats & (PBG_S_HAP_K | PBG_S_HAP_EHHS);
    L.segcap = segcap;
    L.seg = take((uint32_t)segcap * 8 * mask_words);
    L.var = take(0);
    L.planecap = planes ? n * (segcap / 64) : 0;
    L.plane = take((uint32_t)L.planecap * 8);
    L.diff = take(zero ? (uint32_t)(n * ((n + 63) / 64)) * 8 : 0);   // row j: ceil(n / 64) words
    L.acc = take((stats & (PBG_S_NUCDIV | PBG_S_HAP_DXY)) ? (uint32_t)(np * np * 4) : 0);
    L.amin = take((stats & PBG_S_HAP_DXY) ? (uint32_t)(np * np * 4) : 0);
    L.bins = take((stats & (PBG_S_SFS | PBG_S_DIV_POP | PBG_S_HAP_K | PBG_S_HAP_EHHS))
                      ? (uint32_t)((np + 1) * (sfs_stride + 2) * 4)   // + one scratch slice (haplo histogram)
                      : 0);
    L.rbuf = take((stats & PBG_S_ZNS) ? (uint32_t)np * 4 : 0);   // ZnS: variable sites per population
    L.r2lds = 0;                                                   // (r^2 tables: window_zns_kernel)
    L.r2 = take(0);
    L.bytes = b + 16;
    return L;
}

template <int RB>
__global__ __launch_bounds__(64) void window_stats_kernel(DevParams P, DevTables T, const void *__restrict__ rows,
                                                          uint32_t n_rows, uint32_t n_win, StatsArgs A) {
    using M = typename RowMask<RB>::T;
    constexpr uint64_t NW = sizeof(M) / 8;   // pool words per mask
    extern __shared__ __align__(16) unsigned char sm[];
    // XCD-aware order: the dispatcher deals workgroups round-robin over the 8 XCDs, so block b
    // runs on XCD b % 8; giving XCD x the contiguous windows [x * per, (x + 1) * per) keeps
    // neighbouring (overlapping) windows on one L2, which then serves their shared rows once
    const uint32_t per = (n_win + 7) / 8;
    const uint32_t w = n_win >= 64 ? (blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;
    if (w >= n_win) return;
    const WinLds &L = A.lds;
    const uint32_t segcap = (uint32_t)L.segcap;
    M *s_seg = reinterpret_cast<M *>(sm + L.seg);
    uint64_t *s_plane = reinterpret_cast<uint64_t *>(sm + L.plane);
    uint64_t *s_zero = reinterpret_cast<uint64_t *>(sm + L.diff);   // [v][u / 64] bit u % 64: v and u do not differ
    int32_t *s_acc = reinterpret_cast<int32_t *>(sm + L.acc);
    int32_t *s_amin = reinterpret_cast<int32_t *>(sm + L.amin);
    int32_t *s_bins = reinterpret_cast<int32_t *>(sm + L.bins);
    int32_t *s_vc = reinterpret_cast<int32_t *>(sm + L.rbuf);
    double *s_r2 = reinterpret_cast<double *>(sm + L.r2);
    __shared__ int32_t s_misc[4];

    const int n = P.n, np = P.npops;
    const int lane = threadIdx.x;
    const uint32_t stats = A.stats;
    const int64_t wb = A.wins[w].beg, we = A.wins[w].end > A.wins[w].beg ? A.wins[w].end : A.wins[w].beg;
    const bool ld_ws = (stats & (PBG_S_OMEGA | PBG_S_WALL)) != 0;  // window_ld_kernel reads the seg list
    for (int i = lane; i < L.r2lds; i += 64) s_r2[i] = T.r2[i];

    // ---- pass over the rows: counted total, ordered compaction of the segregating rows (the
    // first segcap into LDS)
    constexpr int R = 16 / RB;
    const uint4 *rw = reinterpret_cast<const uint4 *>(rows);
    const int64_t c0 = wb / R, c1 = (we + R - 1) / R;
    auto load_word = [&](int64_t c) -> uint4 {
        uint4 q = make_uint4(0, 0, 0, 0);
        if (c < c1) {
            if ((c + 1) * R <= (int64_t)n_rows) {
                q = rw[c];
            } else {   // the batch's last, partial 16-byte word: no read past its rows
                uint32_t wd[4] = {0, 0, 0, 0};
                const unsigned char *rb = reinterpret_cast<const unsigned char *>(rows) + c * 16;
                for (int x = 0; (int64_t)c * 16 + x < (int64_t)n_rows * RB && x < 16; x += 2)
                    wd[x >> 2] |= (uint32_t)(*reinterpret_cast<const uint16_t *>(rb + x)) << (8 * (x & 3));
                q = make_uint4(wd[0], wd[1], wd[2], wd[3]);
            }
        }
        return q;
    };
    // seg rows of word c (in window): bit mask + types; `store` gets (index, types)
    // the window's 16-byte words in groups of kLoadAhead per lane: a group's loads are issued
    // together, so the dependent compaction steps wait on one memory latency per group
#ifndef PBG_WIN_AHEAD
#define PBG_WIN_AHEAD 4
#endif
    constexpr int kLoadAhead = PBG_WIN_AHEAD;
    // PBG_BOUNDS: a pool store at word idx must lie in the slice [sl_lo, sl_lo + sl_len) the
    // window took (compact's second pass writes there; its first pass writes LDS)
    uint64_t sl_lo = 0, sl_len = 0;
    auto pool_ok = [&](uint64_t idx) { return PBG_POOL_OK(A, idx, sl_lo, sl_len); };
    (void)pool_ok;
    (void)sl_len;
    auto compact = [&](M *dst, uint32_t cap, bool count_sites, int &my_counted) -> uint32_t {
        const bool in_pool = dst != s_seg;
        (void)in_pool;
        uint32_t S = 0;
        uint4 qa[kLoadAhead];
        for (int64_t cg = c0; cg < c1; cg += 64 * kLoadAhead) {
#pragma unroll
        for (int u = 0; u < kLoadAhead; ++u) qa[u] = load_word(cg + 64 * u + lane);
#pragma unroll
        for (int u = 0; u < kLoadAhead; ++u) {
            const int64_t cb = cg + 64 * u;
            if (cb >= c1) break;   // wave-uniform
            const int64_t c = cb + lane;
            const uint4 q = qa[u];
            M t[R];
            uint32_t segm = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t i = c * R + r;
                bool cnt, sg;
                row_in_word<RB>(q, r, t[r], cnt, sg);
                const bool in = c < c1 && i >= wb && i < we;
                if (count_sites) my_counted += (in && cnt) ? 1 : 0;
                segm |= (in && sg) ? (1u << r) : 0u;
            }
            const uint32_t ls = (uint32_t)__popc(segm);
            const uint32_t incl = wave_incl_scan_s(ls);
            uint32_t j = S + incl - ls;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if ((segm >> r) & 1u) {
                    if (j < cap && (!in_pool || pool_ok(sl_lo + (uint64_t)j * NW))) dst[j] = t[r];
                    ++j;
                }
            S += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        }
        return S;
    };
    int my_counted = 0;
    const uint32_t S = compact(s_seg, segcap, true, my_counted);
    const int num_sites = wave_sum(my_counted);
    const int nwords = S > 0 ? (int)((S + 63) / 64) : 1;
    const bool sums = (stats & (PBG_S_NUCDIV | PBG_S_HAP_DXY)) != 0;
    const bool zbits = (stats & (PBG_S_HAP_K | PBG_S_HAP_EHHS)) != 0;
    // calc_nucdiv's population-pair sums (below) come from per-site derived counts instead of
    // sample pairs when no pair's u16 difference can wrap (S < 2^16), every pair v < u of the
    // sums has pop(v) <= pop(u) (populations in id order), no minimum is asked for and it is the
    // shorter loop
    bool fast_sums = false;
    if (sums && !(stats & PBG_S_HAP_DXY) && P.pops_ordered && S < 65536u) {
        int cost_pairs = 0;
        for (int a = 0; a < np; ++a)
            for (int b = a; b < np; ++b) {
                const int na = P.pop_start[a + 1] - P.pop_start[a], nb = P.pop_start[b + 1] - P.pop_start[b];
                cost_pairs += (na * nb + 63) / 64;
            }
        fast_sums = np * (np + 1) / 2 * (int)((S + 63) / 64) <= cost_pairs * nwords;
    }
    // bitplanes: every sample's, or only calc_nhaps' (its local indices stay below pop_nmax)
    const int plane_n = ((stats & (PBG_S_DIV_IND | PBG_S_HAP_DXY | PBG_S_TREE)) || ((stats & PBG_S_NUCDIV) && !fast_sums))
                            ? n
                            : (zbits ? min(n, P.pop_nmax) : 0);
    const bool need_planes = plane_n > 0;
    // pool slice (u64 words): [seg rows: S masks][bitplanes: n*nwords, when they outgrow LDS]
    // [omega / Wall lists: np*S masks]
    const bool over = S > segcap;
    M *wsg = nullptr;
    uint64_t *wpl = nullptr;
    if (over || ld_ws) {
        const uint64_t npl = (over && need_planes) ? (uint64_t)n * nwords : 0, nli = ld_ws ? (uint64_t)np * S * NW : 0;
        const uint64_t size = S * NW + npl + nli;
        unsigned long long off = 0;
        if (lane == 0) {
            off = atomicAdd(A.pool_used, (unsigned long long)size);
            if (off + size > A.pool_cap) {
                atomicOr(A.err, 4);
                off = ~0ULL;
            } else {
                A.win_off[2 * w] = off;
                A.win_off[2 * w + 1] = off + S * NW + npl;
            }
        }
        off = __shfl(off, 0, 64);
        if (off == ~0ULL) {   // pool exhausted: reported by pbg_check, this window's outputs unset
            if (lane == 0 && A.seg_count) A.seg_count[w] = 0;
            return;
        }
        wsg = reinterpret_cast<M *>(A.pool + off);
        wpl = A.pool + off + S * NW;
        sl_lo = off;
        sl_len = size;
        __syncthreads();
        if (over) {
            int unused = 0;
            (void)compact(wsg, S, false, unused);   // second pass, only for windows beyond segcap
        } else {
            for (uint32_t j = (uint32_t)lane; j < S; j += 64)
                if (pool_ok(sl_lo + (uint64_t)j * NW)) wsg[j] = s_seg[j];
        }
    }
    __syncthreads();
    auto seg_at = [&](uint32_t j) -> M { return j < segcap ? s_seg[j] : wsg[j]; };

    const pbg_window_out &O = A.out;
    if (lane == 0) {
        if (O.num_sites) O.num_sites[w] = num_sites;
        if (O.segsites) O.segsites[w] = (int)S;
        if (A.seg_count) A.seg_count[w] = (int)S;
    }
    const int npairs = np * (np - 1);

    // ---- bitplanes (hap.seq) and the u16 pairwise-difference matrix
    uint64_t *plane = nullptr;
    if (need_planes) {
        plane = (n * nwords <= L.planecap) ? s_plane : wpl;
        // plane[v*nwords + k] bit b = sample v derived at segregating site 64k+b (hap.seq), rows
        // v < plane_n: one ballot per (word, sample), or, for few sites, lanes over the samples
        // each gathering its bits from the (LDS) rows
        if (nwords == 1 && (int)S * ((plane_n + 63) / 64) < plane_n) {
            for (int v0 = 0; v0 < plane_n; v0 += 64) {
                const int v = v0 + lane;
                if (v < plane_n) {
                    uint64_t m = 0;
                    for (uint32_t j = 0; j < S; ++j) m |= (uint64_t)bit(s_seg[j], v) << j;
                    if (plane != wpl || pool_ok((uint64_t)(plane - A.pool) + (uint64_t)v)) plane[v] = m;
                }
            }
        } else {
            for (int k = 0; k < nwords; ++k) {
                const uint32_t j = (uint32_t)(k * 64 + lane);
                const M t = j < S ? seg_at(j) : M{};
                for (int v = 0; v < plane_n; ++v) {
                    const uint64_t m = __ballot(bit(t, v));
                    if (lane == 0 && (plane != wpl || pool_ok((uint64_t)(plane - A.pool) + (uint64_t)(v * nwords + k))))
                        plane[v * nwords + k] = m;
                }
            }
        }
        __syncthreads();
    }
    // calc_diff_matrix (pop_nucdiv.cpp:242-256): u16 accumulation of XOR popcounts (wraps,
    // Appendix A.7), computed pair by pair from the bitplanes and reduced on the spot:
    //  - calc_nucdiv / calc_minDxy: pair (v, u), v < u, adds to (pop(v), pop(u)) when pop(v) <=
    //    pop(u) -- the reference's i <= j loops (Dxy asymmetry, Appendix A.6).  Integer sums, exact
    //    as the reference's doubles are: per pair of populations, lanes over its sample pairs, a
    //    wave sum (and minimum);
    //  - calc_nhaps: one bit per pair (the samples do not differ), from wave ballots.
    auto pair_diff = [&](int v, int u) -> uint32_t {
        uint32_t d = 0;
        if (v != u)
            for (int k = 0; k < nwords; ++k) d += pc(plane[v * nwords + k] ^ plane[u * nwords + k]);
        return d & 0xFFFFu;
    };
    const int zw = (n + 63) >> 6;   // s_zero words per row
    if (zbits) {   // calc_nhaps: row v bit u (v < u < pop_nmax) = samples v and u do not differ
        const int zn = min(n, P.pop_nmax);
        for (int v = 0; v + 1 < zn; ++v)
            for (int u0 = (v + 1) & ~63; u0 < zn; u0 += 64) {
                const int u = u0 + lane;
                const uint64_t m = __ballot(u > v && u < zn && pair_diff(v, u) == 0);
                if (lane == 0) s_zero[v * zw + (u0 >> 6)] = m;
            }
    }
    if (sums && fast_sums) {
        // pair (a, b): sum over sites of c_a (n_b - c_b) + (n_a - c_a) c_b, a < b, or c_a (n_a - c_a)
        // (c = derived members at the site): the same integers as the sample-pair loop below
        for (int a = 0; a < np; ++a)
            for (int b = a; b < np; ++b) {
                const int na = P.pop_start[a + 1] - P.pop_start[a], nb = P.pop_start[b + 1] - P.pop_start[b];
                const M ma = pop_mask<M>(P, a), mb = pop_mask<M>(P, b);
                int acc = 0;
                for (uint32_t j = (uint32_t)lane; j < S; j += 64) {
                    const M t = seg_at(j);
                    const int ca = (int)pc(t & ma), cb = (int)pc(t & mb);
                    acc += a == b ? ca * (na - ca) : ca * (nb - cb) + (na - ca) * cb;
                }
                acc = wave_sum(acc);
                if (lane == 0) s_acc[a * np + b] = acc;
            }
    } else if (sums) {   // per population pair (a, b), a <= b: lanes over its sample pairs (v, u), v < u
        for (int a = 0; a < np; ++a)
            for (int b = a; b < np; ++b) {
                const int a0 = P.pop_start[a], na = P.pop_start[a + 1] - a0;
                const int b0 = P.pop_start[b], nb = P.pop_start[b + 1] - b0;
                int acc = 0, mn = 65535;   // UINT_MAX narrowed to u16 (A.7)
                for (int q = lane; q < na * nb; q += 64) {
                    const int x = q / nb, y = q - x * nb;
                    const int v = P.pop_member[a0 + x], u = P.pop_member[b0 + y];
                    if (v < u) {
                        const int d = (int)pair_diff(v, u);
                        acc += d;
                        mn = min(mn, d);
                    }
                }
                acc = wave_sum(acc);
                if ((stats & PBG_S_HAP_DXY) && a < b) mn = wave_min(mn);
                if (lane == 0) {
                    s_acc[a * np + b] = acc;
                    if (stats & PBG_S_HAP_DXY) s_amin[a * np + b] = a < b ? mn : 65535;
                }
            }
    }
    if (sums || zbits) __syncthreads();
    if (sums) {
        for (int pr = lane; pr < np * np; pr += 64) {
            const int i = pr / np, j = pr - i * np;
            if (j < i) continue;
            double acc = (double)s_acc[pr];
            if (i != j) {
                acc *= 1.0 / (double)(P.pop_n[i] * P.pop_n[j]);
                const int pi = i * np + (j - (i + 1));
                if ((stats & PBG_S_NUCDIV) && O.dxy) O.dxy[(size_t)w * npairs + pi] = x86nan(acc / num_sites);
                if (stats & PBG_S_HAP_DXY) {
                    if (O.hap_dxy) O.hap_dxy[(size_t)w * npairs + pi] = x86nan(acc);
                    if (O.hap_min) O.hap_min[(size_t)w * npairs + pi] = s_amin[pr];
                }
            } else {
                acc *= 2.0 / (double)(P.pop_n[i] * (P.pop_n[i] - 1));
                if (acc != acc) acc = 0.0;
                if ((stats & PBG_S_NUCDIV) && O.pi) O.pi[(size_t)w * np + i] = x86nan(acc / num_sites);
                if ((stats & PBG_S_HAP_DXY) && O.hap_val) O.hap_val[(size_t)w * np + i] = acc;
            }
        }
    }

    // ---- per-population derived counts of every segregating site (calc_sfs, calc_diverge -o 1):
    // bins[i][freq] by LDS atomics; freq is flipped when the outgroup carries the derived allele
    const int bstride = P.sfs_stride + 2;
    if (stats & (PBG_S_SFS | PBG_S_DIV_POP)) {
        for (int i = lane; i < np * bstride; i += 64) s_bins[i] = 0;
        __syncthreads();
        for (uint32_t j = (uint32_t)lane; j < S; j += 64) {
            const M t = seg_at(j);
            const bool flip = (P.flag & PBG_F_OUTGROUP) && bit(t, A.outidx);
            for (int i = 0; i < np; ++i) {
                const unsigned f = pc(t & pop_mask<M>(P, i));
                const unsigned freq = flip ? (unsigned)(uint16_t)(P.pop_n[i] - (int)f) : f;
                atomicAdd(&s_bins[i * bstride + (int)freq], 1);
            }
        }
        __syncthreads();
    }
    if ((stats & PBG_S_SFS) && lane < np) {
        const int i = lane, nn = P.pop_n[i];
        const int32_t *sfs = s_bins + i * bstride;
        int S_i = 0;
        for (int j = 1; j < nn; ++j) S_i += sfs[j];
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
        if (O.seg_pop) O.seg_pop[(size_t)w * np + i] = S_i;
        if (O.theta_w) O.theta_w[(size_t)w * np + i] = (double)S_i / T.a1[nn];   // Watterson: S / a1[n]
        if (O.sfs_bins)
            for (int j = 0; j < P.sfs_stride; ++j)
                O.sfs_bins[((size_t)w * np + i) * P.sfs_stride + j] = j <= nn ? sfs[j] : 0;
    }
    // ---- diverge -o 1 (lane per population): Fixed (freq == n, u16) and Seg (0 < freq < n)
    if ((stats & PBG_S_DIV_POP) && lane < np) {
        const int i = lane, nn = P.pop_n[i];
        const int32_t *sfs = s_bins + i * bstride;
        int segs = 0;
        for (int j = 1; j < nn; ++j) segs += sfs[j];
        const uint32_t fixed = (uint32_t)(nn >= 0 && nn <= P.sfs_stride ? sfs[nn] : 0) & 0xFFFFu;
        const double pd = (P.flag & PBG_F_SUBSTITUTE) ? (double)fixed / num_sites : (double)(fixed + segs) / num_sites;
        const double v = A.jc ? -0.75 * log(1.0 - pd * (4.0 / 3.0)) : pd;
        if (O.div_fixed) O.div_fixed[(size_t)w * np + i] = (int32_t)fixed;
        if (O.div_seg) O.div_seg[(size_t)w * np + i] = segs;
        if (O.div_pop) O.div_pop[(size_t)w * np + i] = x86nan(v);
    }

    // ---- ld -o 0 (calc_zns, pop_ld.cpp:201-252): per population, the ordered list of the
    // segregating rows variable within it (masked to the population) goes to the pool for
    // window_zns_kernel, with num_snps (variable sites among the first S-1, plus the final
    // unconditional increment)
    const uint64_t zreg = A.zstride / (uint64_t)np;   // ZnS list words per population region
    if ((stats & PBG_S_ZNS) && A.zstride && (uint64_t)S * NW > zreg) {
        // the plan's stride was sized for shorter windows (a window list changed in place):
        // report it (pbg_check -> PBG_E_RANGE) instead of writing past the region
        if (lane == 0) atomicOr(A.err, 4);
        if (lane < np) {
            A.var_count[(size_t)w * np + lane] = 0;
            A.zoff[(size_t)w * np + lane] = 0;
            A.ld_ns[(size_t)w * np + lane] = 0;
        }
    } else if ((stats & PBG_S_ZNS) && A.zstride) {
        // lists at fixed places: one pass per population writes the list and counts it
        for (int i = 0; i < np; ++i) {
            const M pm = pop_mask<M>(P, i);
            const int nn = P.pop_n[i], mf = A.min_freq;
            const uint64_t off = (uint64_t)w * A.zstride + (uint64_t)i * zreg;
            M *vl = reinterpret_cast<M *>(A.zlist + off);
            uint32_t V = 0;
            int lastvar = 0;
            for (uint32_t c0 = 0; c0 < S; c0 += 64) {
                const uint32_t j = c0 + (uint32_t)lane;
                M t{};
                bool v = false;
                if (j < S) {
                    t = seg_at(j) & pm;
                    const int m = (int)pc(t);
                    v = m >= mf && m <= nn - mf;
                    if (j == S - 1) lastvar = v ? 1 : 0;
                }
                const uint64_t bm = __ballot(v);
                const uint32_t vi = V + (uint32_t)__popcll(bm & ((1ULL << lane) - 1));
                if (v && PBG_POOL_OK(A, off + (uint64_t)vi * NW, off, zreg)) vl[vi] = t;
                V += (uint32_t)__popcll(bm);
            }
            // num_snps: variable sites among the first S-1, plus the final increment
            if (lane == (S ? (int)((S - 1) & 63u) : 0)) {   // the lane that saw row S-1 knows lastvar
                const int ns = S >= 1 ? (int)V - lastvar + 1 : 0;
                A.var_count[(size_t)w * np + i] = (int)V;
                A.zoff[(size_t)w * np + i] = off;
                A.ld_ns[(size_t)w * np + i] = ns;
                if (O.ld_snps) O.ld_snps[(size_t)w * np + i] = ns;
            }
        }
    } else if (stats & PBG_S_ZNS) {
        // counts first (one pool allocation per window), then the lists
        uint32_t tot = 0;
        for (int i = 0; i < np; ++i) {
            const M pm = pop_mask<M>(P, i);
            const int nn = P.pop_n[i], mf = A.min_freq;
            uint32_t V = 0;
            int lastvar = 0;
            for (uint32_t c0 = 0; c0 < S; c0 += 64) {
                const uint32_t j = c0 + (uint32_t)lane;
                bool v = false;
                if (j < S) {
                    const int m = (int)pc(seg_at(j) & pm);
                    v = m >= mf && m <= nn - mf;
                    if (j == S - 1) lastvar = v ? 1 : 0;
                }
                V += (uint32_t)__popcll(__ballot(v));
            }
            lastvar = wave_sum(lastvar);
            if (lane == 0) {
                const int ns = S >= 1 ? (int)V - lastvar + 1 : 0;
                s_vc[i] = (int)V;
                A.var_count[(size_t)w * np + i] = (int)V;
                A.ld_ns[(size_t)w * np + i] = ns;
                if (O.ld_snps) O.ld_snps[(size_t)w * np + i] = ns;
            }
            tot += V;
        }
        unsigned long long off = 0;
        if (lane == 0 && tot) {
            off = atomicAdd(A.pool_used, (unsigned long long)(tot * NW));
            if (off + tot * NW > A.pool_cap) {
                atomicOr(A.err, 4);
                off = ~0ULL;
            }
        }
        off = __shfl(off, 0, 64);
        __syncthreads();
        for (int i = 0; i < np; ++i) {
            const M pm = pop_mask<M>(P, i);
            const int nn = P.pop_n[i], mf = A.min_freq;
            const uint32_t Vi = (uint32_t)s_vc[i];
            if (lane == 0) A.zoff[(size_t)w * np + i] = off;
            if (off == ~0ULL) {   // pool exhausted: the chain sums nothing (err reported)
                if (lane == 0) A.var_count[(size_t)w * np + i] = 0;
                continue;
            }
            M *vl = reinterpret_cast<M *>(A.pool + off);
            uint32_t V = 0;
            for (uint32_t c0 = 0; c0 < S; c0 += 64) {
                const uint32_t j = c0 + (uint32_t)lane;
                M t{};
                bool v = false;
                if (j < S) {
                    t = seg_at(j) & pm;
                    const int m = (int)pc(t);
                    v = m >= mf && m <= nn - mf;
                }
                const uint64_t bm = __ballot(v);
                const uint32_t vi = V + (uint32_t)__popcll(bm & ((1ULL << lane) - 1));
                if (v && PBG_POOL_OK(A, off + (uint64_t)vi * NW, off, (uint64_t)Vi * NW)) vl[vi] = t;
                V += (uint32_t)__popcll(bm);
            }
            off += Vi * NW;
        }
    }

    // ---- diverge -o 0 (lane per sample): u16 accumulation of derived counts
    if (stats & PBG_S_DIV_IND)
        for (int v = lane; v < n; v += 64) {
            uint32_t d = 0;
            for (int k = 0; k < nwords; ++k) d += pc(plane[v * nwords + k]);
            const double pd = (double)(d & 0xFFFF) / num_sites;
            const double x = A.jc ? -0.75 * log(1.0 - pd * (4.0 / 3.0)) : pd;
            if (O.div_ind) O.div_ind[(size_t)w * n + v] = x86nan(x);
        }
    // ---- tree: treeData's diff_matrix (calc_diff_matrix, pop_tree.cpp:472-494), u16 values;
    //      taxon 0 is the reference (row = the sample's derived count), taxon i+1 sample i
    if ((stats & PBG_S_TREE) && O.tree_diff) {
        const int nt = n + 1;
        int32_t *td = O.tree_diff + (size_t)w * nt * nt;
        for (int pr = lane; pr < nt * nt; pr += 64) {
            const int a = pr / nt, b = pr - a * nt;
            int32_t v = 0;
            if (a != b && (a == 0 || b == 0)) {
                const int smp = a + b - 1;
                uint32_t d = 0;
                for (int k = 0; k < nwords; ++k) d += pc(plane[smp * nwords + k]);
                v = (int32_t)(d & 0xFFFF);
            } else if (a != b) {
                v = (int32_t)pair_diff(a - 1, b - 1);
            }
            td[pr] = v;
        }
    }

    // ---- haplo K / Kdiv and EHHS: one population at a time, lanes over its samples / sites
    if (stats & (PBG_S_HAP_K | PBG_S_HAP_EHHS))
        for (int i = 0; i < np; ++i) {
            const int nelem = P.pop_n[i];
            int nh = 1;
            double hdiv = 1.0;
            int32_t *b = s_bins + i * bstride;    // sample ids of the population (<= sfs_stride - 1)
            int32_t *hist = s_bins + np * bstride;   // scratch slice after the populations'
            if (nelem > 1) {
                // b[c] = global id of the population's c-th sample (pop_member: ascending ids)
                const int a0 = P.pop_start[i];
                for (int j = lane; j < nelem; j += 64) hist[j] = 0;
                // calc_nhaps's merge loop (pop_haplo.cpp:221-231), local indices j, k into the
                // global diff matrix (A.11).  Step j only reads b[j], final once steps < j are
                // done, and each b[k], k > j: the k's of one step run across lanes.
                auto zero_bit = [&](int j, int k) -> bool { return (s_zero[j * zw + (k >> 6)] >> (k & 63)) & 1u; };
                if (nelem <= 64) {   // b in registers: lane k holds b[k]
                    int bk = lane < nelem ? (int)P.pop_member[a0 + lane] : 0;
                    for (int j = 0; j < nelem - 1; j++) {
                        const int bj = __builtin_amdgcn_readlane(bk, j);
                        const uint64_t zrow = s_zero[j * zw];
                        if (lane > j && lane < nelem && ((zrow >> lane) & 1u) && bk > bj) bk = j;
                    }
                    __syncthreads();
                    // f_j = #{q : b[q] == j}, j < nelem: an LDS histogram
                    if (lane < nelem && bk >= 0 && bk < nelem) atomicAdd(&hist[bk], 1);
                } else {
                    for (int j = lane; j < nelem; j += 64) b[j] = (int)P.pop_member[a0 + j];
                    __syncthreads();
                    for (int j = 0; j < nelem - 1; j++) {
                        const int bj = b[j];
                        for (int k = j + 1 + lane; k < nelem; k += 64)
                            if (zero_bit(j, k) && b[k] > bj) b[k] = j;
                        __syncthreads();
                    }
                    for (int q = lane; q < nelem; q += 64)
                        if (b[q] >= 0 && b[q] < nelem) atomicAdd(&hist[b[q]], 1);
                }
                __syncthreads();
                int my_nh = 0, my_ff = 0;
                for (int j = lane; j < nelem; j += 64) {
                    const int f = hist[j];
                    my_nh += f > 0 ? 1 : 0;
                    my_ff += f * f;
                }
                nh = wave_sum(my_nh);
                const int ff = wave_sum(my_ff);
                const double sh = (double)(ff) / (double)(nelem * nelem);
                hdiv = 1.0 - ((1.0 - sh) * (double)(nelem / (nelem - 1)));
                __syncthreads();   // hist / b reused by the next population
            }
            if (stats & PBG_S_HAP_K) {
                if (lane == 0) {
                    if (O.nhaps) O.nhaps[(size_t)w * np + i] = nh;
                    if (O.hap_val) O.hap_val[(size_t)w * np + i] = x86nan(1.0 - hdiv);
                }
            } else {
                double e;
                if (nelem < 4) {
                    e = __longlong_as_double(0x7FF8000000000000LL);
                } else {
                    // max multiplicity among non-singleton partitions, ties -> smallest value
                    // (std::list sort + unique + remove, pop_haplo.cpp:273-313): lanes over the
                    // candidate sites, then a (count desc, value asc) reduction across lanes
                    const M pm = pop_mask<M>(P, i);
                    int best = 0;
                    M max_site{};
                    for (uint32_t j = (uint32_t)lane; j < S; j += 64) {
                        const M pt = seg_at(j) & pm;
                        const unsigned f = pc(pt);
                        if (!(f > 1 && (int)f < nelem - 1)) continue;
                        int cnt = 0;
                        for (uint32_t q = 0; q < S; q++) cnt += (seg_at(q) & pm) == pt;
                        const int part_count = cnt + 1;
                        if (part_count > best || (part_count == best && pt < max_site)) {
                            best = part_count;
                            max_site = pt;
                        }
                    }
                    for (int o = 32; o > 0; o >>= 1) {
                        const int ob = __shfl_xor(best, o, 64);
                        const M os = shfl_xor_mask(max_site, o);
                        if (ob > best || (ob == best && os < max_site)) {
                            best = ob;
                            max_site = os;
                        }
                    }
                    const unsigned popf = pc(max_site);
                    const int pn = nelem;
                    const double sh = (1.0 - ((double)((int)(popf * popf) + ((pn - (int)popf) * (pn - (int)popf))) / (pn * pn))) *
                                      (double)(pn / (pn - 1));
                    e = hdiv / (1.0 - sh);
                }
                if (lane == 0 && O.hap_val) O.hap_val[(size_t)w * np + i] = e;
            }
        }
    (void)s_misc;
}

// Serial LD chains, one lane per chain (pop_ld.cpp:254-458), reading the ordered segregating
// lists window_stats_kernel copied into the pool.  Lanes of a wave belong to
// different windows, so the dependent double additions of 64 chains overlap.
template <class M>
__global__ __launch_bounds__(kBlockThreads) void window_ld_kernel(DevParams P, DevTables T, uint32_t n_win, StatsArgs A) {
    constexpr uint64_t NW = sizeof(M) / 8;
    __shared__ double s_r2[4096];
    const int np = P.npops;
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
        const int S = A.seg_count[w];
        const M *seg = reinterpret_cast<const M *>(A.pool + A.win_off[2 * w]);
        int ns[PBG_MAX_POPS], cong[PBG_MAX_POPS], part[PBG_MAX_POPS], nu[PBG_MAX_POPS];
        for (int j = 0; j < np; j++) ns[j] = cong[j] = part[j] = nu[j] = 0;
        M *uniq = reinterpret_cast<M *>(A.pool + A.win_off[2 * w + 1]);   // np slices of S
        M last_type{};
        for (int i = 0; i < S; i++) {
            const M t = seg[i];
            for (int j = 0; j < np; j++) {
                const M pm = pop_mask<M>(P, j);
                const M type = t & pm;
                const M comp = ~t & pm;
                M *u = uniq + (uint64_t)j * (uint64_t)S;
                if (nonzero(type) && type < pm) {
                    if (ns[j] == 0) {
                        if (PBG_POOL_OK(A, A.win_off[2 * w + 1] + ((uint64_t)j * S + nu[j]) * NW, A.win_off[2 * w + 1],
                                        (uint64_t)np * S * NW))
                            u[nu[j]] = type;
                        ++nu[j];
                        last_type = type;
                        ns[j]++;
                    } else {
                        if (type == last_type || comp == last_type) {
                            cong[j]++;
                            bool seen = false;
                            for (int q = 0; q < nu[j]; q++) seen |= (u[q] == type) || (u[q] == comp);
                            if (!seen) {
                                if (PBG_POOL_OK(A, A.win_off[2 * w + 1] + ((uint64_t)j * S + nu[j]) * NW,
                                                A.win_off[2 * w + 1], (uint64_t)np * S * NW))
                                    u[nu[j]] = type;
                                ++nu[j];
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
    const int S = A.seg_count[w];
    const M *seg = reinterpret_cast<const M *>(A.pool + A.win_off[2 * w]);
    const int nn = P.pop_n[i], np1 = nn + 1, mf = A.min_freq;
    const M pm = pop_mask<M>(P, i);
    const double *r2p = r2tab + T.r2_off[i];
    auto variable = [&](unsigned m) { return (int)m >= mf && (int)m <= nn - mf; };
    int ns = 0;
    double val = 0.0;
    {   // calc_omegamax pop_ld.cpp:254-373 (sums accumulate across partitions, A.8)
        if (S >= 1) {
            int V = 0;
            M *vt = reinterpret_cast<M *>(A.pool + A.win_off[2 * w + 1] + (uint64_t)i * (uint64_t)S * NW);
            for (int j = 0; j < S; j++) {
                const M t = seg[j] & pm;
                if (variable(pc(t))) {
                    if (j < S - 1) ++ns;
                    if (PBG_POOL_OK(A, A.win_off[2 * w + 1] + ((uint64_t)i * S + V) * NW, A.win_off[2 * w + 1],
                                    (uint64_t)np * S * NW))
                        vt[V] = t;
                    ++V;
                }
            }
            ++ns;
            auto r2 = [&](int a, int b) -> double {   // a < b; 0 beyond the variable sites
                if (b >= V) return 0.0;
                const M ta = vt[a], tb = vt[b];
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

// ZnS (calc_zns, pop_ld.cpp:201-252) as producer / consumer.  The reference's value of a
// (window, population) chain is one sequential double sum of r^2 over every pair (a, b), a < b,
// of the population's variable sites, in pair order: V(V-1)/2 dependent additions.  A workgroup
// owns C consecutive chains and has 64 + 16 G C threads.  Wave 0 is the adder: lane c keeps chain
// c's running double and, per round, adds the chain's next 16 values in pair order from an LDS
// ring (eight 16-byte reads issued a round ahead, then 16 register adds: the dependent chain
// never waits on another lane).  Producer group (c, h) (16 lanes, h < G = kZnsG) walks chain c a
// row step per round, taking the rounds r with r % G == h: lane j computes r^2 of pair (a, b0 + j) from the popcounts of the two sites' masks and of their
// intersection (the host's r^2 table); lanes past the row's end give +0.0, which leaves the sum
// unchanged, so the adder sees the reference's exact sequence of additions.  Rounds run in
// phases of kZnsR: while the adder sums phase k - 1 from one half of the ring, the producers
// fill the other half with phase k; one workgroup barrier per phase.  A producer first walks the
// phase's kZnsR / G pairs (register arithmetic), then issues all their list reads, then all their
// table reads, so a phase costs two LDS latencies, not 2 kZnsR.
//
// Fast path (every population of at most 26 samples and every list of the workgroup within the
// LDS list capacity): the lists are staged in LDS as one u32 per site, the population-compacted
// mask | popcount << 26, and the r^2 tables sit in LDS with a 0.0 slot past them, so a pair is
// two LDS reads (the row's entry a broadcast), five VALU and the table read.
// Otherwise the raw masks (u64 / two-word) are read from the list buffer in HBM / L2, the table
// from LDS or HBM.
#ifndef PBG_ZNS_EXP
#define PBG_ZNS_EXP 0   // timing experiments only (wrong results): bit 0 producers idle, bit 1 adder idle
#endif
#ifndef PBG_ZNS_SORT
#define PBG_ZNS_SORT 1
#endif
#ifndef PBG_ZNS_PRIO
#define PBG_ZNS_PRIO 3
#endif
// Two 16-lane producer groups per chain (rounds dealt out in turn: group h takes rounds h, h + 2,
// ...): the producers of a workgroup's longest chains had been the slower side of each phase
// (configs[2] statistics 0.2105 -> 0.1975 ms, A/B in one call; four groups: 0.243 ms, fewer chains
// per workgroup, more workgroups than two per CU)
#ifndef PBG_ZNS_GROUPS
#define PBG_ZNS_GROUPS 2
#endif
constexpr int kZnsG = PBG_ZNS_GROUPS;        // 16-lane producer groups per chain
constexpr int kZnsMaxC = 60 / kZnsG;         // chains per workgroup (64 + 16 G C <= 1024 threads)
constexpr int kZnsR = 8;                     // rounds per phase
constexpr int kZnsRingStride = 18;           // doubles per (round, chain): 16 values + 2 pad (LDS banks)

// the sample bits of t inside population mask pm, packed to bit positions 0..pc(pm)-1
__device__ __forceinline__ uint32_t pext32(uint64_t t, uint64_t pm, uint32_t &k) {
    uint32_t out = 0;
    while (pm) {
        const int p = __builtin_ctzll(pm);
        out |= (uint32_t)((t >> p) & 1u) << k;
        ++k;
        pm &= pm - 1;
    }
    return out;
}
__device__ __forceinline__ uint32_t compact32(uint64_t t, uint64_t pm) {
    uint32_t k = 0;
    return pext32(t, pm, k);
}
__device__ __forceinline__ uint32_t compact32(M2 t, M2 pm) {
    uint32_t k = 0;
    const uint32_t lo = pext32(t.lo, pm.lo, k);
    return lo | pext32(t.hi, pm.hi, k);
}
// row-step rounds of a chain of V sites: sum over the V - 1 rows of ceil(row length / 16)
__device__ __forceinline__ long long zns_rounds(int V) {
    const long long N = V > 1 ? V - 1 : 0, q = N / 16, r = N % 16;
    return (q + 1) * (8 * q + r);
}

struct ZnsChain {   // per-chain constants, LDS
    const void *list;   // the chain's raw masks (M) in the list buffer
    int32_t V, np1, r2o, ns;
    int32_t w;
};

template <class M>
__global__ __launch_bounds__(1024) void window_zns_kernel(DevParams P, DevTables T, uint32_t n_win, StatsArgs A,
                                                          int r2_lds, int C, int cap, int compact) {
    extern __shared__ __align__(16) double s_dyn[];
    __shared__ ZnsChain s_ch[kZnsMaxC];
    __shared__ long long s_rounds;
    __shared__ int s_fits;
    const int tid = (int)threadIdx.x, np = P.npops, nthr = (int)blockDim.x;
    const uint32_t nch = n_win * (uint32_t)np;
    const uint32_t ch0 = blockIdx.x * (uint32_t)C;
    // LDS: r^2 tables (+ a 0.0 slot) | ring [2][kZnsR][C][kZnsRingStride] | lists [C][cap] u32
    double *s_r2t = s_dyn;
    const int r2_slots = r2_lds ? ((r2_lds + 2) & ~1) : 0;
    double *s_ring = s_dyn + r2_slots;
    uint32_t *s_lst = reinterpret_cast<uint32_t *>(s_ring + 2 * kZnsR * C * kZnsRingStride);
    const size_t rstride = (size_t)C * kZnsRingStride;   // doubles per round
    if (tid == 0) {
        s_rounds = 0;
        s_fits = compact;
    }
    for (int i = tid; i < r2_lds; i += nthr) s_r2t[i] = T.r2[i];
    if (tid == 0 && r2_lds) s_r2t[r2_lds] = 0.0;
    __syncthreads();
    if (tid < C) {
        const uint32_t ch = ch0 + (uint32_t)tid;
        ZnsChain z{nullptr, 0, 1, 0, 0, 0};
        if (ch < nch) {
            const uint32_t w = ch / (uint32_t)np;
            const int i = (int)(ch - w * (uint32_t)np);
            z.list = (A.zstride ? A.zlist : A.pool) + A.zoff[ch];
            z.V = A.var_count[ch];
            z.np1 = P.pop_n[i] + 1;
            z.r2o = T.r2_off[i];
            z.ns = A.ld_ns[ch];
            z.w = (int)w;
        }
        s_ch[tid] = z;
        atomicMax(reinterpret_cast<unsigned long long *>(&s_rounds), (unsigned long long)zns_rounds(z.V));
        if (z.V > cap) atomicAnd(&s_fits, 0);
    }
    __syncthreads();
    // producer group / adder lane g works on chain s_ord[g]: the workgroup's chains longest first,
    // so the producer waves of the short ones (four consecutive groups each) run out together and
    // skip their remaining phases
    __shared__ int s_ord[kZnsMaxC];
    if (tid < C) {
        int rk = tid;
        if (PBG_ZNS_SORT) {
            const long long rt = zns_rounds(s_ch[tid].V);
            rk = 0;
            for (int c2 = 0; c2 < C; ++c2) {
                const long long r2 = zns_rounds(s_ch[c2].V);
                rk += (r2 > rt || (r2 == rt && c2 < tid)) ? 1 : 0;
            }
        }
        s_ord[rk] = tid;
    }
    const long long nphase = (s_rounds + kZnsR - 1) / kZnsR;
    const bool fast = s_fits != 0 && r2_lds != 0;   // workgroup-uniform
    if (fast) {   // stage the lists compacted: wave v takes chains v, v + (waves), ...
        const int wv = tid >> 6, lane = tid & 63, nwv = nthr >> 6;
        for (int c = wv; c < C; c += nwv) {
            const ZnsChain z = s_ch[c];
            const int i = (int)((ch0 + (uint32_t)c) % (uint32_t)np);
            const M pm = pop_mask<M>(P, i);
            const M *L = reinterpret_cast<const M *>(z.list);
            for (int b = lane; b < z.V; b += 64) {
                const uint32_t m = compact32(L[b], pm);
                s_lst[c * cap + b] = m | (uint32_t)__popc(m) << 26;   // compacted mask | popcount << 26
            }
        }
    }
    __syncthreads();   // the staged lists
    if (tid < 64) {
        // ---- the adder: lane c sums chain c's values in pair order
#if PBG_ZNS_PRIO
        __builtin_amdgcn_s_setprio(PBG_ZNS_PRIO);   // the dependent chain issues ahead of the producers
#endif
        double acc = 0.0;
        const int cg = tid < C ? s_ord[tid] : 0;
        const long long rg_end = tid < C ? zns_rounds(s_ch[cg].V) : 0;   // the chain's rounds
        for (long long k = 0; k <= nphase; ++k) {   // phase k: sum phase k - 1 (the producers write phase k)
            // (a phase past the chain's last round holds only +0.0 or, skipped, nothing: no adds)
            if (k >= 1 && tid < C && (k - 1) * kZnsR < rg_end) {
                const double2 *rg = reinterpret_cast<const double2 *>(s_ring + (size_t)((k - 1) & 1) * kZnsR * rstride +
                                                                      (size_t)tid * kZnsRingStride);
                double2 v[8];
#pragma unroll
                for (int x = 0; x < 8; ++x) v[x] = rg[x];
#pragma unroll
                for (int r = 0; r < kZnsR; ++r) {   // the next round's values are read before this round's adds
                    double2 nv[8];
                    if (r + 1 < kZnsR) {
#pragma unroll
                        for (int x = 0; x < 8; ++x) nv[x] = rg[(size_t)(r + 1) * (rstride / 2) + x];
                    }
                    // the next round's eight reads stay ahead of this round's sixteen adds (left to
                    // itself, the scheduler sank them to one or two adds before their first use)
                    __builtin_amdgcn_sched_barrier(0);
#if !(PBG_ZNS_EXP & 2)   // (timing experiment 2: no adds)
#pragma unroll
                    for (int x = 0; x < 8; ++x) {
                        acc += v[x].x;
                        acc += v[x].y;
                    }
#endif
                    __builtin_amdgcn_sched_barrier(0);
                    if (r + 1 < kZnsR) {
#pragma unroll
                        for (int x = 0; x < 8; ++x) v[x] = nv[x];
                    }
                }
            }
            __syncthreads();
        }
        if (tid < C && ch0 + (uint32_t)cg < nch) {
            const ZnsChain z = s_ch[cg];
            double val = 0.0;
            if (A.seg_count[z.w] >= 1) val = acc * (2.0 / (z.ns * (z.ns - 1)));
            if (A.out.ld_val) A.out.ld_val[ch0 + (uint32_t)cg] = x86nan(val);
        }
        return;
    }
    // ---- the producers: group c = (tid - 64) / 16 walks chain c, lane j takes pair (a, b0 + j)
    const int p = tid - 64, j = p & 15, g = (p >> 4) / kZnsG, h = (p >> 4) % kZnsG, c = s_ord[g];
    const ZnsChain z = s_ch[c];
    const long long my_rounds = zns_rounds(z.V);
    const int V = z.V, V1 = z.V - 1, np1 = z.np1, r2o = z.r2o, vm = max(V1, 0);
    int a = 0, b0 = 1;
    auto step = [&]() {   // the next row step of the chain's pair walk
        b0 += 16;
        const bool nxt = b0 >= V;
        a += nxt ? 1 : 0;
        b0 = nxt ? a + 1 : b0;
    };
    for (int x = 0; x < h; ++x) step();   // group h takes rounds h, h + G, ...
    const uint32_t *lst = s_lst + c * cap;
    const uint32_t np1sq = (uint32_t)(np1 * np1);
    const M *L = reinterpret_cast<const M *>(z.list);
    const double *tab = r2_lds ? s_r2t : T.r2;
    for (long long k = 0; k <= nphase; ++k) {
        // (a wave whose four chains are all past their last round skips the phase)
        if (k < nphase && !(PBG_ZNS_EXP & 1) && __ballot(k * kZnsR < my_rounds) != 0) {   // (exp 1: producers idle)
            double *out = s_ring + (size_t)(k & 1) * kZnsR * rstride + (size_t)g * kZnsRingStride + j;
            // the phase's pairs first (pure VALU), then every load of the phase in flight at once
            constexpr int R = kZnsR / kZnsG;   // this group's rounds of the phase
            int pa[R], pb[R];
            bool ok[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                pa[r] = a;
                pb[r] = b0 + j;
                ok[r] = (a < V1) & (pb[r] < V);
#pragma unroll
                for (int x = 0; x < kZnsG; ++x) step();
            }
            double v[R];
            if (fast) {
                uint32_t ea[R], eb[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    ea[r] = lst[min(pa[r], vm)];   // clamped, not selected: no branch (unused when !ok)
                    eb[r] = lst[min(pb[r], vm)];
                }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int idx = r2o + (int)(__umul24(ea[r] >> 26, np1sq) + __umul24(eb[r] >> 26, (uint32_t)np1)) +
                                    __popc(ea[r] & eb[r] & 0x03FFFFFFu);
                    v[r] = s_r2t[ok[r] ? idx : r2_lds];
                }
            } else if (V > 1) {   // (a chain without pairs may have no list at all)
                M ta[R], tb[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    ta[r] = L[min(pa[r], vm)];
                    tb[r] = L[min(pb[r], vm)];
                }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double x = tab[r2o + ((int)pc(ta[r]) * np1 + (int)pc(tb[r])) * np1 + (int)pc(ta[r] & tb[r])];
                    v[r] = ok[r] ? x : 0.0;
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = 0.0;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) out[(size_t)(r * kZnsG + h) * rstride] = v[r];
        }
        __syncthreads();
    }
}

template __global__ void window_stats_kernel<2>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<4>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<8>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);
template __global__ void window_stats_kernel<16>(DevParams, DevTables, const void *, uint32_t, uint32_t, StatsArgs);

hipError_t launch_window_stats(int rb, const DevParams &P, const DevTables &T, const void *rows, uint32_t n_rows,
                               uint32_t n_win, const StatsArgs &A, hipStream_t stream, int n_cu) {
    if (n_win == 0) return hipSuccess;
    // window_stats_kernel's XCD-aware order: 8 * ceil(n_win / 8) workgroups (the extra exit at once)
    const dim3 g(n_win >= 64 ? (n_win + 7) / 8 * 8 : n_win), b(64);
    const size_t lds = A.lds.bytes;
    switch (rb) {
        case 2: hipLaunchKernelGGL(window_stats_kernel<2>, g, b, lds, stream, P, T, rows, n_rows, n_win, A); break;
        case 4: hipLaunchKernelGGL(window_stats_kernel<4>, g, b, lds, stream, P, T, rows, n_rows, n_win, A); break;
        case 8: hipLaunchKernelGGL(window_stats_kernel<8>, g, b, lds, stream, P, T, rows, n_rows, n_win, A); break;
        default: hipLaunchKernelGGL(window_stats_kernel<16>, g, b, lds, stream, P, T, rows, n_rows, n_win, A); break;
    }
    if (A.stats & PBG_S_ZNS) {
        int r2_total = 0, max_pop = 0;
        for (int i = 0; i < P.npops; ++i) {
            r2_total += (P.pop_n[i] + 1) * (P.pop_n[i] + 1) * (P.pop_n[i] + 1);
            max_pop = std::max(max_pop, P.pop_n[i]);
        }
        const int r2_lds = r2_total <= 4608 ? r2_total : 0;   // <= 36 KB of LDS
        const uint32_t chains = n_win * (uint32_t)P.npops;
        // C chains per workgroup (64 + 16 G C threads): two workgroups per CU when the chains allow
        // it (two barrier domains interleave on a CU: 0.229 against 0.233 ms of statistics with
        // one), and as many as the LDS budget holds with lists of up to 256 sites
        const size_t budget = 75 * 1024;   // LDS per workgroup: two per CU
        const size_t tab = (size_t)(r2_lds ? ((r2_lds + 2) & ~1) : 0) * 8;
        const size_t per_chain = (size_t)2 * kZnsR * kZnsRingStride * 8 + 256 * 4;
        const uint32_t cfit = budget > tab + per_chain ? (uint32_t)((budget - tab) / per_chain) : 1u;
        const int C = (int)std::max<uint32_t>(1u, std::min<uint32_t>(std::min<uint32_t>((uint32_t)kZnsMaxC, cfit),
                                                                      (chains + 2 * n_cu - 1) / std::max(1, 2 * n_cu)));
        const size_t fixed = tab + (size_t)2 * kZnsR * C * kZnsRingStride * 8;
        int cap = budget > fixed ? (int)std::min<size_t>(4096, (budget - fixed) / ((size_t)C * 4)) & ~7 : 0;
        // fast path: compacted 26-bit masks (populations of at most 26 samples)
        const int compact = (max_pop <= 26 && r2_lds && cap >= 16) ? 1 : 0;
        if (!compact) cap = 0;
        const size_t lds = fixed + (size_t)C * cap * 4;
        const dim3 g((chains + C - 1) / C), b(64 + 16 * kZnsG * C);
        if (rb == 16)
            hipLaunchKernelGGL(window_zns_kernel<M2>, g, b, lds, stream, P, T, n_win, A, r2_lds, C, cap, compact);
        else
            hipLaunchKernelGGL(window_zns_kernel<uint64_t>, g, b, lds, stream, P, T, n_win, A, r2_lds, C, cap, compact);
    }
    const uint32_t ld = A.stats & (PBG_S_OMEGA | PBG_S_WALL);
    if (ld) {
        if (ld != PBG_S_OMEGA && ld != PBG_S_WALL) return hipErrorInvalidValue;
        const uint32_t chains = (ld == PBG_S_WALL) ? n_win : n_win * (uint32_t)P.npops;
        const dim3 g((chains + kBlockThreads - 1) / kBlockThreads);
        if (rb == 16) hipLaunchKernelGGL(window_ld_kernel<M2>, g, dim3(kBlockThreads), 0, stream, P, T, n_win, A);
        else hipLaunchKernelGGL(window_ld_kernel<uint64_t>, g, dim3(kBlockThreads), 0, stream, P, T, n_win, A);
    }
    return hipGetLastError();
}

}  // namespace pbg
