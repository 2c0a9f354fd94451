// api.cpp -- the C-ABI of include/popbam_gpu.h: context, resident-batch launches
// (pbg_call_sites / pbg_window_stats / pbg_check), the synthetic generator and pbg_format.
// Streamed runs over host batches (pbg_stream_*, pbg_run) are in stream.cpp.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "pbg_ctx.h"


namespace {

thread_local std::string g_create_error;

int fail(pbg_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    else g_create_error = msg;
    return code;
}

}  // namespace

int pbg::ctx_fail(pbg_ctx *c, int code, const std::string &msg) { return fail(c, code, msg); }

namespace {

#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail((ctx), PBG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

// rms of call_base (popbam.cpp:292) for k keys with sum mapQ^2 = rmsq: the reference's float
// division, sqrtf and (unsigned long long)(x + 0.499)
uint32_t rms_of(uint32_t rmsq, int k) {
    const float f = (float)rmsq / (float)k;
    return (uint32_t)((double)std::sqrt(f) + 0.499);
}
// smallest sum mapQ^2 (mapQ <= 255) whose rms passes qfilter with k keys, or ~0 when none does
uint32_t rms_threshold(int k, int min_rmsQ, int min_depth, int max_depth) {
    if (k < 1 || k < min_depth || k > max_depth) return 0xFFFFFFFFu;
    uint32_t lo = 0, hi = (uint32_t)k * 65025u;   // rms is monotone in rmsq
    if ((int)rms_of(hi, k) < min_rmsQ) return 0xFFFFFFFFu;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if ((int)rms_of(mid, k) >= min_rmsQ) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

int row_bytes_for(int n) { return n <= 14 ? 2 : n <= 30 ? 4 : n <= 62 ? 8 : 16; }

template <class T>
hipError_t upload(T **dst, const std::vector<T> &v) {
    hipError_t e = hipMalloc((void **)dst, std::max<size_t>(1, v.size()) * sizeof(T));
    if (e != hipSuccess) return e;
    if (v.empty()) return hipSuccess;
    return hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}


}  // namespace

namespace pbg {
extern const int kBuildKind_call, kBuildKind_stats;
}

namespace {
// errmod_tables.bin beside this library (written by `make`, pbg_host.h)
std::string tables_path() {
    Dl_info info;
    if (!dladdr((void *)&pbg_create, &info) || !info.dli_fname) return std::string();
    std::string p = info.dli_fname;
    const size_t sl = p.rfind('/');
    return (sl == std::string::npos ? std::string(".") : p.substr(0, sl)) + "/errmod_tables.bin";
}
}  // namespace

extern "C" {

int pbg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *pbg_last_error(const pbg_ctx *ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int pbg_row_bytes(const pbg_ctx *ctx) { return ctx ? ctx->row_bytes : 0; }
int pbg_k_bytes(const pbg_ctx *ctx) { return ctx ? (ctx->dp.k16 ? 2 : 1) : 0; }
int pbg_sfs_stride(const pbg_ctx *ctx) { return ctx ? ctx->dp.sfs_stride : 0; }

int pbg_create(pbg_ctx **out, int device, const pbg_params *p) {
    if (!out || !p) return fail(nullptr, PBG_E_ARG, "null argument");
    *out = nullptr;
    if (p->n_samples < 1 || p->n_samples > PBG_MAX_SAMPLES)
        return fail(nullptr, PBG_E_ARG, "n_samples must be in [1, 126]");
    if (p->n_pops < 1 || p->n_pops > PBG_MAX_POPS) return fail(nullptr, PBG_E_ARG, "n_pops must be in [1, 64]");
    if (p->max_depth < 0 || p->max_depth > 65535) return fail(nullptr, PBG_E_ARG, "max_depth must be in [0, 65535]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, PBG_E_NODEV, "no HIP device visible (libpopbam_gpu has no CPU path)");
    if (device < 0 || device >= ndev) return fail(nullptr, PBG_E_NODEV, "device index out of range");
    pbg_ctx *c = new pbg_ctx();
    c->device = device;
    c->params = *p;
    c->row_bytes = row_bytes_for(p->n_samples);
    pbg::DevParams &d = c->dp;
    d.n = p->n_samples;
    d.npops = p->n_pops;
    for (int i = 0; i < PBG_MAX_POPS; ++i) {
        d.pop_mask[i] = i < p->n_pops ? p->pop_mask[i] : 0;
        d.pop_mask_hi[i] = i < p->n_pops && p->n_samples > 64 ? p->pop_mask_hi[i] : 0;
        d.pop_n[i] = i < p->n_pops ? p->pop_n[i] : 0;
    }
    d.min_depth = p->min_depth;
    d.max_depth = p->max_depth;
    d.min_rmsQ = p->min_rmsQ;
    d.min_snpQ = p->min_snpQ;
    d.min_mapQ = p->min_mapQ & 0xff;
    d.min_baseQ = p->min_baseQ & 0xff;
    d.flag = p->flag;
    d.k16 = p->max_depth > 255 ? 1 : 0;
    // population of each sample: assign_pops gives every sample one population (popbam.cpp:145-171)
    for (int v = 0; v < PBG_MAX_SAMPLES; ++v) d.sample_pop[v] = -1;
    for (int i = 0; i < p->n_pops; ++i)
        for (int v = 0; v < p->n_samples; ++v)
            if (((v < 64 ? p->pop_mask[i] >> v : d.pop_mask_hi[i] >> (v - 64)) & 1)) {
                if (d.sample_pop[v] >= 0) {
                    delete c;
                    return fail(nullptr, PBG_E_ARG, "population masks overlap");
                }
                d.sample_pop[v] = (int8_t)i;
            }
    {   // samples grouped by population (window statistics: per-population-pair loops)
        int at = 0;
        for (int i = 0; i < p->n_pops; ++i) {
            d.pop_start[i] = (int16_t)at;
            for (int v = 0; v < p->n_samples; ++v)
                if (d.sample_pop[v] == i) d.pop_member[at++] = (uint8_t)v;
        }
        for (int i = p->n_pops; i <= PBG_MAX_POPS; ++i) d.pop_start[i] = (int16_t)at;
        d.pop_nmax = 0;
        d.pops_ordered = 1;
        int last = -1;   // largest member id of the populations so far
        for (int i = 0; i < p->n_pops; ++i) {
            const int a0 = d.pop_start[i], a1 = d.pop_start[i + 1];
            d.pop_nmax = std::max(d.pop_nmax, a1 - a0);
            if (a1 > a0) {
                if (d.pop_member[a0] < last) d.pops_ordered = 0;
                last = d.pop_member[a1 - 1];
            }
        }
    }
    for (int k = 0; k <= PBG_FAST_MAX; ++k) d.rms_thr[k] = rms_threshold(k, p->min_rmsQ, p->min_depth, p->max_depth);
    d.rmsq_thr[0] = p->min_rmsQ <= 0 ? 0u : 0xFFFFFFFFu;
    for (int k = 1; k <= 16; ++k) d.rmsq_thr[k] = rms_threshold(k, p->min_rmsQ, 1, 1 << 30);
    d.sfs_stride = 1;
    for (int i = 0; i < p->n_pops; ++i) d.sfs_stride = std::max(d.sfs_stride, p->pop_n[i] + 1);
    auto bad = [&](hipError_t e, const char *what) {
        std::string m = std::string(what) + ": " + hipGetErrorString(e);
        pbg_destroy(c);
        return fail(nullptr, PBG_E_HIP, m);
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bad(e, "hipSetDevice");
    if ((e = hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
        return bad(e, "hipDeviceGetAttribute");
    if (c->n_cu < 1) c->n_cu = 1;
    std::vector<double> fk, beta, lhet;
    if (!pbg::load_errmod_tables(tables_path().c_str(), fk, beta, lhet)) pbg::build_errmod_tables(fk, beta, lhet);
    // the scan's reference-only shortcut needs every beta[q][n][c < n] > 0 (q >= 4, n <= PBG_FAST_MAX)
    for (int q = 4; q < 64; ++q)
        for (int nn = 1; nn <= PBG_FAST_MAX; ++nn)
            for (int cc = 0; cc < nn; ++cc)
                if (!(beta[q << 16 | nn << 8 | cc] > 0.0)) {
                    pbg_destroy(c);
                    return fail(nullptr, PBG_E_ARG, "errmod beta table has a non-positive entry");
                }
    if ((e = upload(&c->d_fk, fk)) != hipSuccess) return bad(e, "upload fk");
    if ((e = upload(&c->d_beta, beta)) != hipSuccess) return bad(e, "upload beta");
    if ((e = upload(&c->d_lhet, lhet)) != hipSuccess) return bad(e, "upload lhet");
    {
        std::vector<double> fbeta(pbg::kFbetaSize, 0.0);
        for (uint32_t q = 0; q < 64; ++q)
            for (uint32_t nn = 0; nn < (uint32_t)pbg::kFbetaN; ++nn)
                for (uint32_t cc = 0; cc < 16; ++cc)
                    for (uint32_t w = 0; w < 16; ++w)
                        // q = 0 stays +0.0 (beta's q = 0 plane is never filled, pop_utils.cpp:230):
                        // the register path relies on it for its zero padding words
                        fbeta[pbg::fbeta_index(q, nn, cc, w)] = q ? fk[w] * beta[q << 16 | nn << 8 | cc] : 0.0;
        if ((e = upload(&c->d_fbeta, fbeta)) != hipSuccess) return bad(e, "upload fbeta");
        std::vector<double> lb(pbg::kLbSize, 0.0);
        for (int m = 1; m <= 16; ++m) lb[m] = lb[m - 1] + fk[m - 1];
        for (int d = 3; d <= 16; ++d) {
            double run = 1e300;   // suffix minimum over q' >= q
            for (int q = 63; q >= 4; --q) {
                for (int cc = 0; cc <= d - 2; ++cc) run = std::min(run, beta[q << 16 | d << 8 | cc]);
                lb[17 + (q - 4) * 17 + d] = run;
            }
        }
        if ((e = upload(&c->d_lb, lb)) != hipSuccess) return bad(e, "upload lb");
        std::vector<double> oe(pbg::kOeSize, 0.0);
        for (int q = 4; q < 64; ++q)
            for (int d = 0; d <= 16; ++d) oe[(q - 4) * 17 + d] = beta[q << 16 | d << 8];
        for (int nn = 0; nn <= 16; ++nn)
            for (int kk = 0; kk <= 16; ++kk) oe[60 * 17 + nn * 17 + kk] = lhet[nn << 8 | kk];
        if ((e = upload(&c->d_oe, oe)) != hipSuccess) return bad(e, "upload one-error tables");
        {   // call_scan_kernel's LDS image of the same tables (pbg_common.h ScanTab)
            pbg::ScanTab st{};
            for (int q = 4; q < 64; ++q)
                for (int dd = 3; dd <= 16; ++dd) {
                    const volatile double pe = fk[0] * beta[q << 16 | dd << 8];   // one_error_ref's product
                    st.fpe[(q - 4) * 14 + dd - 3] = (float)pe;
                }
            for (int lev = 0; lev < 15; ++lev)
                for (int dd = 3; dd <= 16; ++dd) {
                    const double b = lb[17 + (4 * lev) * 17 + dd];   // q = 4 + 4 lev: a bound for the level
                    float f = (float)b;
                    if ((double)f > b) f = std::nextafter(f, 0.0f);   // rounded down
                    st.lq[lev * 14 + dd - 3] = f;
                }
            for (int dd = 3; dd <= 16; ++dd) {
                const int idx[4][2] = {{dd, dd - 1}, {dd, 1}, {dd - 1, 0}, {dd - 1, dd - 1}};
                for (int i = 0; i < 4; ++i) {
                    const volatile double h = -4.343 * lhet[idx[i][0] << 8 | idx[i][1]];
                    st.lh[(dd - 3) * 4 + i] = h;
                }
            }
            for (int m = 0; m <= 16; ++m) st.pre[m] = lb[m];
            if ((e = hipMalloc(&c->d_scantab, sizeof(st))) != hipSuccess) return bad(e, "hipMalloc scan tables");
            if ((e = hipMemcpy(c->d_scantab, &st, sizeof(st), hipMemcpyHostToDevice)) != hipSuccess)
                return bad(e, "upload scan tables");
        }
        std::vector<double> bu(60 * 17, 0.0);   // min over q' >= q, c <= d - 1 of beta[q'][d][c]
        for (int dd = 1; dd <= 16; ++dd) {
            double run = 1e300;
            for (int q = 63; q >= 4; --q) {
                for (int cc = 0; cc <= dd - 1; ++cc) run = std::min(run, beta[q << 16 | dd << 8 | cc]);
                bu[(q - 4) * 17 + dd] = run;
            }
        }
        // uniform tasks: het values and the strand-free bound per (d, m class, q); since fk
        // decreases, fk_prefix[m0] + fk_prefix[m1] >= fk_prefix[m0 + m1], so fk_prefix[d] is a
        // lower bound of the per-strand sum whatever the strands
        bool fk_dec = true;   // fk[n] = (1 - depcorr)^n (1 - eta) + eta (pop_utils.cpp:219) decreases
        for (int w = 1; w < 16; ++w) fk_dec = fk_dec && fk[w] <= fk[w - 1];
        for (int i = 0; i < 17 * 3; ++i) d.uni[i] = 255u;
        for (int dd = 1; dd <= 16; ++dd) {
            float h[2];
            for (int t = 0; t < 2; ++t) {   // het m/x with c_hi = 0 / d: (float)(-4.343 lhet), clamped
                const float v = (float)(-4.343 * lhet[dd << 8 | (t ? dd : 0)]);
                h[t] = v < 0.0f ? 0.0f : v;
            }
            const float hm[3] = {h[0], h[1], std::min(h[0], h[1])};
            for (int cls = 0; cls < 3; ++cls) {
                uint32_t qthr = 255u;   // the bound grows with q_min (suffix minimum): first passing q
                for (int q = 63; q >= 4; --q) {
                    const double lbv = lb[dd] * bu[(q - 4) * 17 + dd];
                    if (fk_dec && hm[cls] > 0.0f && lbv * (1.0 - 1e-9) > (double)hm[cls] * (1.0 + 1e-6) + 1e-3) qthr = (uint32_t)q;
                    else break;
                }
                const uint32_t snpq = (uint32_t)(uint64_t)((double)hm[cls] + 0.499) & 0xFFFFu;
                d.uni[dd * 3 + cls] = qthr | snpq << 8;
            }
        }
    }
    // Tajima constants are indexed by population size and built for n = sm->n (pop_sfs.cpp:53-56)
    std::vector<double> a1, a2, e1, e2;
    pbg::build_sfs_constants(p->n_samples, a1, a2, e1, e2);
    const size_t L = a2.size();
    std::vector<double> sfs(4 * L, 0.0);
    std::copy(a1.begin(), a1.end(), sfs.begin());
    std::copy(a2.begin(), a2.end(), sfs.begin() + L);
    std::copy(e1.begin(), e1.end(), sfs.begin() + 2 * L);
    std::copy(e2.begin(), e2.end(), sfs.begin() + 3 * L);
    if ((e = upload(&c->d_sfs, sfs)) != hipSuccess) return bad(e, "upload sfs constants");
    std::vector<double> r2all;
    for (int i = 0; i < p->n_pops; ++i) {
        std::vector<double> t;
        pbg::build_r2_table(std::max(1, p->pop_n[i]), t);
        c->dt.r2_off[i] = (int32_t)r2all.size();
        r2all.insert(r2all.end(), t.begin(), t.end());
    }
    if ((e = upload(&c->d_r2, r2all)) != hipSuccess) return bad(e, "upload r2 tables");
    if ((e = hipMalloc(&c->d_err, sizeof(int))) != hipSuccess) return bad(e, "hipMalloc err");
    if ((e = hipMemset(c->d_err, 0, sizeof(int))) != hipSuccess) return bad(e, "hipMemset err");
    c->dt.fk = c->d_fk;
    c->dt.beta = c->d_beta;
    c->dt.lhet = c->d_lhet;
    c->dt.fbeta = c->d_fbeta;
    c->dt.lb = c->d_lb;
    c->dt.oe = c->d_oe;
    c->dt.scantab = reinterpret_cast<const uint4 *>(c->d_scantab);
    c->dt.a1 = c->d_sfs;
    c->dt.a2 = c->d_sfs + L;
    c->dt.e1 = c->d_sfs + 2 * L;
    c->dt.e2 = c->d_sfs + 3 * L;
    c->dt.r2 = c->d_r2;
    *out = c;
    return PBG_OK;
}

void pbg_destroy(pbg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    pbg::stream_bufs_free(c);
    for (void *p : {(void *)c->d_fk, (void *)c->d_beta, (void *)c->d_lhet, (void *)c->d_sfs, (void *)c->d_r2,
                    (void *)c->d_fbeta, (void *)c->d_lb, (void *)c->d_oe, c->d_scantab, (void *)c->d_err, (void *)c->d_ws, (void *)c->d_wsoff, (void *)c->d_zns,
                    (void *)c->deep.sites, (void *)c->deep.tasks, (void *)c->deep.info, (void *)c->deep.count,
                    (void *)c->deep.blk_cnt, (void *)c->deep.raw, (void *)c->deep.pend,
                    (void *)c->d_segcnt, (void *)c->d_synth})
        if (p) (void)hipFree(p);
    for (auto &t : c->tmpl) (void)hipFree(t.second);
    for (auto *v : {&c->ev, &c->evc})
        for (auto &e : *v) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
    delete c;
}

int pbg_call_sites(pbg_ctx *c, const pbg_pileup *pl, void *rows, uint64_t *cb, void *stream) {
    if (!c || !pl || !rows) return fail(c, PBG_E_ARG, "null argument");
    if (pl->n_sites == 0) return PBG_OK;
    if (!pl->ref || !pl->k || !pl->rmsq || !pl->block_off || !pl->keys) return fail(c, PBG_E_ARG, "null pileup array");
    if (((uintptr_t)pl->keys | (uintptr_t)pl->k | (uintptr_t)pl->rmsq | (uintptr_t)rows) & 15)
        return fail(c, PBG_E_ARG, "keys / k / rmsq / rows must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->device));
    const uint32_t nblk = (pl->n_sites + pbg::kSiteBlock - 1) / pbg::kSiteBlock;
    const int64_t hint = c->cap_hint_keys;
    c->cap_hint_keys = -1;
    if (cb && (hint >= 0 || c->cap_key != (const void *)pl->block_off || c->cap_sites != pl->n_sites)) {
        // LDS staging capacity of the consensus-word kernel: the mean round plus six standard
        // deviations (Poisson-like), bounded by what one CU can give a workgroup; rounds above
        // it read HBM directly.  The batch's keys are block_off[nblk] - block_off[0] (offsets may
        // be absolute, include/popbam_gpu.h); a streamed chunk passes its count from the host
        uint64_t total = 0;
        if (hint >= 0) {
            total = (uint64_t)hint;
        } else {
            uint64_t ends[2] = {0, 0};
            HIPCHK(c, hipMemcpyAsync(&ends[0], pl->block_off, sizeof(uint64_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
            HIPCHK(c, hipMemcpyAsync(&ends[1], pl->block_off + nblk, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                     (hipStream_t)stream));
            HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
            total = ends[1] >= ends[0] ? ends[1] - ends[0] : 0;
        }
        // keys staged per round = keys of kBlockThreads consecutive (position, sample) tasks
        const double mean = (double)total / ((double)pl->n_sites * c->dp.n) * pbg::kBlockThreads;
        uint32_t cap = (uint32_t)(mean + 6.0 * std::sqrt(mean) + 64.0);
        cap = (cap + 63) & ~63u;
        const uint32_t max_cap = (uint32_t)((48 * 1024 - pbg::call_sites_lds_bytes(c->dp.n, 0)) / 4);
        c->cap_val = std::min(std::max(cap, 256u), max_cap);
        c->cap_key = hint >= 0 ? nullptr : pl->block_off;   // a hinted chunk's slot pointer repeats
        c->cap_sites = pl->n_sites;
    }
    const uint32_t cap = c->cap_val;
    // queues: positions (worst case all), parked info bytes (n per position), per-block queue
    // regions of 3/16 of the block's tasks (+32) for the rows-only pipeline (segregating
    // positions cluster queued tasks; the rest is computed by the overflow kernel); the
    // consensus-word pipeline's deep queue shares the task array
    if (c->deep_sites_cap < pl->n_sites || c->deep_info_cap < (size_t)pl->n_sites * c->dp.n) {
        for (void *p : {(void *)c->deep.sites, (void *)c->deep.tasks, (void *)c->deep.info, (void *)c->deep.blk_cnt,
                        (void *)c->deep.raw, (void *)c->deep.pend})
            if (p) HIPCHK(c, hipFree(p));
        c->deep.blk_cnt = nullptr;
        c->deep.raw = nullptr;
        c->deep.pend = nullptr;
        c->deep.sites = nullptr;
        c->deep.tasks = nullptr;
        c->deep.info = nullptr;
        c->deep_sites_cap = c->deep_info_cap = 0;
        const size_t ntask = (size_t)pl->n_sites * c->dp.n;
        const uint32_t blk_cap = (uint32_t)(pbg::kSiteBlock * c->dp.n * 3 / 16 + 32);
        const size_t tcap = std::max<size_t>((size_t)nblk * blk_cap, std::min<size_t>(ntask / 32 + 65536, 0xFFFFFFFFu));
        HIPCHK(c, hipMalloc((void **)&c->deep.sites, (size_t)pl->n_sites * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc((void **)&c->deep.tasks, tcap * sizeof(pbg::DeepTask)));
        HIPCHK(c, hipMalloc((void **)&c->deep.info, ntask + 64));   // + slack: the scan's fold reads whole dwords
        HIPCHK(c, hipMalloc((void **)&c->deep.pend, (size_t)nblk * sizeof(uint64_t)));
        c->deep.task_cap = (uint32_t)std::min<size_t>(tcap, 0xFFFFFFFFu);
        c->deep.blk_cap = blk_cap;
        HIPCHK(c, hipMalloc((void **)&c->deep.blk_cnt, (size_t)nblk * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc((void **)&c->deep.raw, (size_t)nblk * blk_cap * 3 * sizeof(uint4)));
        c->deep_sites_cap = pl->n_sites;
        c->deep_info_cap = ntask;
        // allocated lengths, for the PBG_BOUNDS store checks
        c->deep.raw_n = c->deep.raw_chk = (uint64_t)nblk * blk_cap * 3;
        c->deep.info_n = c->deep.info_chk = ntask;
        c->deep.tasks_n = c->deep.tasks_chk = c->deep.task_cap;
        c->deep.blk_n = c->deep.blk_chk = nblk;
        c->deep.sites_n = c->deep.sites_chk = pl->n_sites;
    }
    if (!c->deep.count) HIPCHK(c, hipMalloc((void **)&c->deep.count, 4 * sizeof(uint32_t)));
    hipEvent_t e0 = nullptr, e1 = nullptr, c0 = nullptr, c1 = nullptr;
    if (c->timing) {
        if (c->ev_used == c->ev.size()) {
            hipEvent_t a, b, x, y;
            HIPCHK(c, hipEventCreate(&a));
            HIPCHK(c, hipEventCreate(&b));
            HIPCHK(c, hipEventCreate(&x));
            HIPCHK(c, hipEventCreate(&y));
            c->ev.emplace_back(a, b);
            c->evc.emplace_back(x, y);
        }
        e0 = c->ev[c->ev_used].first;
        e1 = c->ev[c->ev_used].second;
        c0 = c->evc[c->ev_used].first;
        c1 = c->evc[c->ev_used].second;
        ++c->ev_used;
        HIPCHK(c, hipEventRecord(c0, (hipStream_t)stream));
    }
    uint32_t shrink = 0;
    pbg::DeepBufs D = c->deep;
    D.rows_div = D.words_div = 1;
#ifdef PBG_BOUNDS
    // positive controls of the bounds build: PBG_BOUNDS_SELFTEST names the class whose checked
    // range is cut (keys: the batch's last chunk; queue / info / block: half the array; deep: all
    // of it; rows / words: half the batch; pool: pbg_window_stats), so correct kernels trip that
    // class's check
    if (const char *st = std::getenv("PBG_BOUNDS_SELFTEST")) {
        const std::string m = st;
        if (m == "1" || m == "keys") shrink = 8u;
        else if (m == "queue") D.raw_chk = D.raw_n / 2;
        else if (m == "info") D.info_chk = D.info_n / 2;
        else if (m == "deep") D.tasks_chk = 0;
        else if (m == "block") D.blk_chk = D.blk_n / 2;
        else if (m == "rows") D.rows_div = 2;
        else if (m == "words") D.words_div = 2;
    }
#endif
    if (cb && c->scan_compact) return fail(c, PBG_E_ARG, "compact pieces carry no keys for reference-only tasks: no consensus words");
    const pbg::Batch B{pl->n_sites, pl->ref, pl->k, pl->rmsq, pl->block_off, pl->keys, c->d_err, c->scan_masked, c->scan_compact,
                       shrink};
    HIPCHK(c, pbg::launch_call_sites(c->row_bytes, c->dp, c->dt, B, cap, rows, cb, c->d_err, D,
                                     (hipStream_t)stream, e0, e1, c->n_cu));
    if (c1) HIPCHK(c, hipEventRecord(c1, (hipStream_t)stream));
    return PBG_OK;
}

const char *pbg_build_info(void) {
    const int kind = std::max({(int)PBG_BUILD_KIND, pbg::kBuildKind_call, pbg::kBuildKind_stats});
    return kind == 2 ? "experiment" : kind == 1 ? "bounds" : "product";
}

int pbg_check(pbg_ctx *c, void *stream) {
    if (!c) return fail(c, PBG_E_ARG, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
    int herr = 0;
    HIPCHK(c, hipMemcpy(&herr, c->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (!herr) return PBG_OK;
    HIPCHK(c, hipMemset(c->d_err, 0, sizeof(int)));
    if (herr & 4) return fail(c, PBG_E_RANGE, "statistics workspace exhausted (windows with very many segregating sites)");
    if (herr & 8) return fail(c, PBG_E_BATCH, "a kernel loaded keys outside [block_off[0], block_off[last]) (PBG_BOUNDS build)");
    if (herr & pbg::kErrQueue) return fail(c, PBG_E_BATCH, "a queue record was stored outside its block's region of the queue (PBG_BOUNDS build)");
    if (herr & pbg::kErrDeep) return fail(c, PBG_E_BATCH, "a deep-task entry was stored outside the task list (PBG_BOUNDS build)");
    if (herr & pbg::kErrInfo) return fail(c, PBG_E_BATCH, "an info byte was stored outside the info array (PBG_BOUNDS build)");
    if (herr & pbg::kErrRow) return fail(c, PBG_E_BATCH, "a row was stored outside the batch's rows (PBG_BOUNDS build)");
    if (herr & pbg::kErrBlock) return fail(c, PBG_E_BATCH, "a block's pending mask / queue count / overflow entry was stored out of range (PBG_BOUNDS build)");
    if (herr & pbg::kErrWords) return fail(c, PBG_E_BATCH, "a consensus word was stored outside the batch's words (PBG_BOUNDS build)");
    if (herr & pbg::kErrCompact) return fail(c, PBG_E_BATCH, "a compact piece flagged a task that is not reference-only (1..32 keys on an upper-case A/C/G/T reference base)");
    if (herr & pbg::kErrPool) return fail(c, PBG_E_BATCH, "a statistics workspace store fell outside its pool slice (PBG_BOUNDS build)");
    if (herr & 2) return fail(c, PBG_E_BATCH, "synthetic batch needs more keys than keys_cap");
    return fail(c, PBG_E_BATCH, "pileup block_off disagrees with k[]");
}

int pbg_set_kernel_timing(pbg_ctx *c, int on) {
    if (!c) return fail(c, PBG_E_ARG, "null argument");
    c->timing = on != 0;
    c->ev_used = 0;
    return PBG_OK;
}

int pbg_kernel_time(pbg_ctx *c, double *ms_total, uint32_t *launches) {
    if (!c || !ms_total || !launches) return fail(c, PBG_E_ARG, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    double tot = 0.0;
    for (size_t i = 0; i < c->ev_used; ++i) {
        HIPCHK(c, hipEventSynchronize(c->ev[i].second));
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev[i].first, c->ev[i].second));
        tot += ms;
    }
    *ms_total = tot;
    *launches = (uint32_t)c->ev_used;
    return PBG_OK;
}

int pbg_call_time(pbg_ctx *c, double *ms_total, uint32_t *launches) {
    if (!c || !ms_total || !launches) return fail(c, PBG_E_ARG, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    double tot = 0.0;
    for (size_t i = 0; i < c->ev_used; ++i) {
        HIPCHK(c, hipEventSynchronize(c->evc[i].second));
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->evc[i].first, c->evc[i].second));
        tot += ms;
    }
    *ms_total = tot;
    *launches = (uint32_t)c->ev_used;
    return PBG_OK;
}

int pbg_window_stats(pbg_ctx *c, const void *rows, uint32_t n_rows, const pbg_window *wins, uint32_t n_win,
                     const pbg_stat_opts *o, const pbg_window_out *out, void *stream) {
    if (!c || !rows || !wins || !o || !out) return fail(c, PBG_E_ARG, "null argument");
    if (n_win == 0) return PBG_OK;
    if ((uintptr_t)rows & 15) return fail(c, PBG_E_ARG, "rows must be 16-byte aligned");
    {
        const uint32_t ld = o->stats & (PBG_S_ZNS | PBG_S_OMEGA | PBG_S_WALL);
        if (ld & (ld - 1)) return fail(c, PBG_E_ARG, "at most one of ZnS / omega / Wall per call (shared outputs)");
    }
    HIPCHK(c, hipSetDevice(c->device));
    pbg::StatsArgs A{};
    A.pool_div = 1;
#ifdef PBG_BOUNDS
    if (const char *st = std::getenv("PBG_BOUNDS_SELFTEST"))
        if (std::string(st) == "pool") A.pool_div = 2;   // positive control of the pool store checks
#endif
    A.stats = o->stats;
    A.min_freq = o->min_freq;
    A.outidx = o->outidx;
    A.jc = o->jc;
    A.wins = wins;
    A.out = *out;
    // statistics workspace: a pool the windows take slices of on the device (windows with more
    // than kSegCap segregating rows, omega / Wall lists, ZnS lists).  Sized from the window list
    // (worst case, at most kPoolMax words); the plan is cached per device window list, so
    // steady-state calls do not synchronise.
    const bool ld_ws = (o->stats & (PBG_S_OMEGA | PBG_S_WALL)) != 0;
    const int n = c->dp.n, np = c->dp.npops;
    const uint64_t mw = c->row_bytes == 16 ? 2 : 1;
    bool known = false;
    uint64_t zstride = 0;
    int segcap = pbg::kSegCap;
    for (const auto &pl : c->plans)
        if (pl.wins == (const void *)wins && pl.n_win == n_win && pl.n_rows == n_rows && pl.stats == o->stats) {
            known = true;
            zstride = pl.zstride;
            segcap = pl.segcap;
        }
    if (!known) {
        std::vector<pbg_window> hw(n_win);
        HIPCHK(c, hipMemcpyAsync(hw.data(), wins, n_win * sizeof(pbg_window), hipMemcpyDeviceToHost,
                                 (hipStream_t)stream));
        HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
        uint64_t worst = 0, maxlen = 0;
        for (uint32_t i = 0; i < n_win; ++i) {
            if (hw[i].beg < 0 || hw[i].end < hw[i].beg || (uint32_t)hw[i].end > n_rows)
                return fail(c, PBG_E_RANGE, "window outside the row range");
            maxlen = std::max<uint64_t>(maxlen, (uint64_t)(hw[i].end - hw[i].beg));
        }
        // segregating rows each window keeps in LDS: short windows need few, and a smaller slice
        // leaves room for more waves per CU (1 kb windows at 96 samples: 64 rows, 1 KB of masks);
        // windows with more spill to the pool
        segcap = maxlen <= 2048 ? 64 : maxlen <= 8192 ? 128 : pbg::kSegCap;
        for (uint32_t i = 0; i < n_win; ++i) {
            const uint64_t len = (uint64_t)(hw[i].end - hw[i].beg);
            // words: masks are mw words each (two for 16-byte rows)
            if (ld_ws || len > (uint64_t)segcap) worst += mw * len + (uint64_t)n * (len / 64 + 1) + (ld_ws ? mw * np * len : 0);
            if (o->stats & PBG_S_ZNS) worst += mw * np * len;
        }
        constexpr uint64_t kPoolMax = 512ull << 20;   // words (4 GiB)
        const uint64_t want = std::max<uint64_t>(1024, std::min(worst, kPoolMax));
        if (want * 8 > c->ws_cap) {
            if (c->d_ws) HIPCHK(c, hipFree(c->d_ws));
            c->d_ws = nullptr;
            HIPCHK(c, hipMalloc(&c->d_ws, want * 8));
            c->ws_cap = want * 8;
        }
        if ((size_t)n_win * 16 + (size_t)n_win * np * 8 + 8 > c->wsoff_cap) {   // win_off | zoff | pool_used
            if (c->d_wsoff) HIPCHK(c, hipFree(c->d_wsoff));
            c->d_wsoff = nullptr;
            c->wsoff_cap = (size_t)n_win * 16 + (size_t)n_win * np * 8 + 8;
            HIPCHK(c, hipMalloc(&c->d_wsoff, c->wsoff_cap));
        }
        // seg_count [n_win] | var_count [n_win*np] | ld_ns [n_win*np]
        const size_t segcnt_bytes = (size_t)n_win * (1 + 2 * (size_t)np) * 4;
        if (segcnt_bytes > c->segcnt_cap) {
            if (c->d_segcnt) HIPCHK(c, hipFree(c->d_segcnt));
            c->d_segcnt = nullptr;
            HIPCHK(c, hipMalloc((void **)&c->d_segcnt, segcnt_bytes));
            c->segcnt_cap = segcnt_bytes;
        }
        // ZnS lists at fixed places (no pool allocation in the kernel) when windows are of
        // (nearly) one length: n_win * npops * maxlen words, at most twice the exact need
        if (o->stats & PBG_S_ZNS) {
            uint64_t need = 0;
            for (uint32_t i = 0; i < n_win; ++i) need += mw * np * (uint64_t)(hw[i].end - hw[i].beg);
            const uint64_t zs = mw * np * std::max<uint64_t>(maxlen, 1);
            if ((uint64_t)n_win * zs <= std::max<uint64_t>(2 * need, 1 << 20) && (uint64_t)n_win * zs <= kPoolMax) {
                zstride = zs;
                if ((uint64_t)n_win * zs * 8 > c->zns_cap) {
                    if (c->d_zns) HIPCHK(c, hipFree(c->d_zns));
                    c->d_zns = nullptr;
                    HIPCHK(c, hipMalloc((void **)&c->d_zns, (size_t)n_win * zs * 8));
                    c->zns_cap = (size_t)n_win * zs * 8;
                }
            }
        }
        if (c->plans.size() >= 16) c->plans.erase(c->plans.begin());
        c->plans.push_back({wins, n_win, n_rows, o->stats, zstride, segcap});
    }
    A.pool = c->d_ws;
    A.pool_cap = c->ws_cap / 8;
    A.win_off = c->d_wsoff;
    A.zoff = c->d_wsoff + 2 * (size_t)n_win;
    A.pool_used = reinterpret_cast<unsigned long long *>(c->d_wsoff + 2 * (size_t)n_win + (size_t)n_win * np);
    A.err = c->d_err;
    HIPCHK(c, hipMemsetAsync(A.pool_used, 0, 8, (hipStream_t)stream));
    A.zlist = c->d_zns;
    A.zstride = zstride;
    A.seg_count = c->d_segcnt;
    A.var_count = c->d_segcnt + n_win;
    A.ld_ns = c->d_segcnt + n_win + (size_t)n_win * np;
    A.lds = pbg::stats_lds_layout(n, np, c->dp.sfs_stride, o->stats, 0, (int)mw, segcap);
    if (A.lds.bytes > 64 * 1024) return fail(c, PBG_E_ARG, "statistics need more LDS than a workgroup has");
    HIPCHK(c, pbg::launch_window_stats(c->row_bytes, c->dp, c->dt, rows, n_rows, n_win, A, (hipStream_t)stream, c->n_cu));
    return PBG_OK;
}

uint64_t pbg_synth_max_keys(const pbg_ctx *c, const pbg_synth_spec *sp) {
    if (!c || !sp) return 0;
    const int dmax = std::min(2 * sp->mean_depth, c->dp.max_depth);
    return (uint64_t)sp->n_sites * (uint64_t)c->dp.n * (uint64_t)std::max(dmax, 0);
}

int pbg_synth_pileup(pbg_ctx *c, const pbg_synth_spec *sp, uint8_t *ref, void *k, uint32_t *rmsq, uint64_t *block_off,
                     uint16_t *keys, uint64_t keys_cap, uint64_t *n_keys, void *stream) {
    if (!c || !sp || !ref || !k || !rmsq || !block_off || (!keys && keys_cap)) return fail(c, PBG_E_ARG, "null argument");
    if (sp->mean_depth < 1 || sp->mean_depth > 32) return fail(c, PBG_E_ARG, "mean_depth must be in [1, 32]");
    if (((uintptr_t)keys | (uintptr_t)k | (uintptr_t)rmsq | (uintptr_t)ref) & 15)
        return fail(c, PBG_E_ARG, "keys / k / rmsq / ref must be 16-byte aligned");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const uint16_t *tmpl = nullptr;
    for (auto &t : c->tmpl)
        if (t.first == sp->seed) tmpl = t.second;
    if (!tmpl) {   // first use of this seed: build its table and wait for it (every stream may read it)
        constexpr size_t kTmplCache = 8;   // tables kept per context (2 MB each)
        if (c->tmpl.size() >= kTmplCache) {   // evict the oldest once no launch can still read it
            HIPCHK(c, hipDeviceSynchronize());
            HIPCHK(c, hipFree(c->tmpl.front().second));
            c->tmpl.erase(c->tmpl.begin());
        }
        uint16_t *t = nullptr;
        HIPCHK(c, hipMalloc((void **)&t, pbg::kTmplSize * sizeof(uint16_t)));
        hipError_t e = pbg::launch_synth_tmpl(sp->seed, t, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {   // never cache a table that was not built
            (void)hipFree(t);
            return fail(c, PBG_E_HIP, std::string("synthetic template table: ") + hipGetErrorString(e));
        }
        c->tmpl.emplace_back(sp->seed, t);   // cached only once built
        tmpl = t;
    }
    const size_t need = pbg::synth_scratch_words(sp->n_sites) * 8;
    if (need > c->synth_cap) {
        if (c->d_synth) HIPCHK(c, hipFree(c->d_synth));
        c->d_synth = nullptr;
        HIPCHK(c, hipMalloc((void **)&c->d_synth, need));
        c->synth_cap = need;
    }
    HIPCHK(c, pbg::launch_synth(c->dp, sp->seed, sp->contig, sp->mean_depth, sp->pos0, sp->n_sites, ref, k, rmsq,
                                block_off, keys, keys_cap, c->d_synth, tmpl, c->d_err, s));
    if (n_keys) {
        const uint32_t nblk = (sp->n_sites + pbg::kSiteBlock - 1) / pbg::kSiteBlock;
        HIPCHK(c, hipMemcpyAsync(n_keys, block_off + nblk, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        int rc = pbg_check(c, stream);
        if (rc) return rc;
    }
    return PBG_OK;
}

long pbg_format(const pbg_ctx *c, const pbg_cmd *cmd, const pbg_window_out *ho, uint32_t n_win, const int32_t *wbeg,
                const int32_t *wend, char *out, size_t cap, size_t *needed) {
    if (!c || !cmd || !ho || !wbeg || !wend || (!out && cap)) return fail(const_cast<pbg_ctx *>(c), PBG_E_ARG, "null argument");
    const int n = c->dp.n, np = c->dp.npops, npairs = std::max(1, np * (np - 1));
    std::string text;
    pbg::WindowHost wh;
    auto take = [](auto *src, size_t off, size_t cnt) {
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(src)>>;
        return src ? std::vector<T>(src + off, src + off + cnt) : std::vector<T>(cnt, T());
    };
    for (uint32_t i = 0; i < n_win; ++i) {
        wh.beg = wbeg[i];
        wh.end = wend[i];
        wh.num_sites = ho->num_sites ? ho->num_sites[i] : 0;
        wh.segsites = ho->segsites ? ho->segsites[i] : 0;
        wh.pi = take(ho->pi, (size_t)i * np, np);
        wh.dxy = take(ho->dxy, (size_t)i * npairs, npairs);
        wh.td = take(ho->td, (size_t)i * np, np);
        wh.fwh = take(ho->fwh, (size_t)i * np, np);
        wh.ld_snps = take(ho->ld_snps, (size_t)i * np, np);
        wh.ld_val = take(ho->ld_val, (size_t)i * np, np);
        wh.ld_q = take(ho->ld_q, (size_t)i * np, np);
        wh.div_ind = take(ho->div_ind, (size_t)i * n, n);
        wh.div_fixed = take(ho->div_fixed, (size_t)i * np, np);
        wh.div_seg = take(ho->div_seg, (size_t)i * np, np);
        wh.div_pop = take(ho->div_pop, (size_t)i * np, np);
        wh.nhaps = take(ho->nhaps, (size_t)i * np, np);
        wh.hap_val = take(ho->hap_val, (size_t)i * np, np);
        wh.hap_dxy = take(ho->hap_dxy, (size_t)i * npairs, npairs);
        wh.hap_min = take(ho->hap_min, (size_t)i * npairs, npairs);
        wh.tree_diff = take(ho->tree_diff, (size_t)i * (n + 1) * (n + 1), (size_t)(n + 1) * (n + 1));
        if (cmd->cmd == PBG_CMD_SFS && (cmd->output & 1) && ho->seg_pop && ho->theta_w && ho->sfs_bins) {
            wh.seg_pop = take(ho->seg_pop, (size_t)i * np, np);
            wh.theta_w = take(ho->theta_w, (size_t)i * np, np);
            wh.sfs_bins.assign(np, {});
            for (int p = 0; p < np; ++p)
                wh.sfs_bins[p] = take(ho->sfs_bins, ((size_t)i * np + p) * c->dp.sfs_stride, (size_t)c->dp.pop_n[p] + 1);
        }
        pbg::format_window(text, *cmd, n, np, c->dp.flag, wh);
    }
    if (needed) *needed = text.size() + 1;
    if (text.size() + 1 > cap) return fail(const_cast<pbg_ctx *>(c), PBG_E_RANGE, "output buffer too small");
    std::memcpy(out, text.c_str(), text.size() + 1);
    return (long)text.size();
}

}  // extern "C"
