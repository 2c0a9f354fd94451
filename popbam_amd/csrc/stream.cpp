// stream.cpp -- streamed runs over HOST pileup batches (pbg_stream_*) and pbg_run on top of them.
//
// The reference's window loop (main_<cmd>, e.g. pop_nucdiv.cpp:47-124) re-fetches and re-piles the
// reads of every window (bam_fetch + bam_plbuf_push per window, pop_nucdiv.cpp:57-125) and calls
// each position on the host inside the pileup callback.  Here the host side of the callback hands
// over the region's key batch in pieces, in position order, as its walk produces them:
//
//   pbg_stream_push(piece)   split into chunks; per chunk, alternating between two device slots:
//                              host  pageable piece -> pinned staging (threaded memcpy), or
//                                    nothing when the caller's buffers are pinned
//                              copy stream     staging / caller buffers -> slot (async H2D)
//                              compute stream  pbg_call_sites(slot) -> the region's rows
//                            so the copy of chunk i+1 runs under the call of chunk i;
//   pbg_stream_finish()      every command's windows over the region's rows (pbg_window_stats,
//                            window lists kept per context by content, so their plans survive
//                            across runs), results to the host, print_<stat> text.
//
// Slots, staging, streams, the rows buffer and the window lists belong to the context and are
// reused by the next stream, so a steady state of pbg_run calls allocates nothing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "pbg_ctx.h"

struct pbg_stream {
    pbg_ctx *c = nullptr;
    std::vector<pbg_cmd> cmds;
    int32_t pos0 = 0;
    uint32_t n_sites = 0;
    uint32_t pushed = 0;
    uint32_t chunk = 0;
    bool words = false;             // a `snp -o 0` command: consensus words are kept
    bool finished = false;
    int rc = PBG_OK;                // sticky first error
    std::vector<uint8_t> href;      // reference bytes of the region (snp printing)
    std::vector<std::string> text;  // per command, after pbg_stream_finish
    pbg_stream_prof prof{};
    std::vector<int> ev_kind;       // per used event pair of c->sb.ev: 0 H2D, 1 call
    int cur = 0;                    // next slot
};

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

int fail(pbg_ctx *c, int code, const std::string &m) { return pbg::ctx_fail(c, code, m); }
#define HIPCHK(ctx, expr) PBG_HIPCHK(ctx, expr)

int row_bytes_of(const pbg_ctx *c) { return c->row_bytes; }

// The chunk's reference has runs of lower-case / N bases (every 16th position sampled; more
// than 1 in 64 of them not upper-case A/C/G/T): POPBAM compares the reference case-sensitively
// (SURVEY Appendix A.5), so every called task there leaves the scan's reference-only test and
// the scan is told to settle its list mid-block (Batch::masked)
bool masked_reference(const uint8_t *ref, uint32_t n) {
    uint32_t odd = 0, seen = 0;
    for (uint32_t i = 0; i < n; i += 16, ++seen) {
        const uint8_t b = ref[i] & 0x7F;
        odd += (b != 'A' && b != 'C' && b != 'G' && b != 'T') ? 1u : 0u;
    }
    return seen && odd * 64u > seen;
}

// pageable caller buffers -> pinned staging: the byte ranges of all jobs split evenly over up
// to 8 threads (one memcpy stream per thread reaches a fraction of the host's bandwidth)
struct CopyJob {
    void *dst;
    const void *src;
    size_t n;
};
void par_copy(const std::vector<CopyJob> &jobs) {
    size_t total = 0;
    for (const auto &j : jobs) total += j.n;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned nt = (unsigned)std::min<size_t>(std::min(8u, hw), std::max<size_t>(1, total / (4u << 20)));
    auto part = [&](size_t lo, size_t hi) {   // bytes [lo, hi) of the jobs' concatenation
        size_t base = 0;
        for (const auto &j : jobs) {
            const size_t a = std::max(lo, base), b = std::min(hi, base + j.n);
            if (a < b) std::memcpy((char *)j.dst + (a - base), (const char *)j.src + (a - base), b - a);
            base += j.n;
        }
    };
    if (nt <= 1) {
        part(0, total);
        return;
    }
    const size_t per = (total + nt - 1) / nt;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(part, std::min(total, t * per), std::min(total, (t + 1) * per));
    part(0, std::min(total, per));
    for (auto &t : th) t.join();
}

bool is_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: not an error worth keeping
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

void free_slot(pbg::StreamSlot &s) {
    for (void *p : {(void *)s.d_ref, s.d_k, (void *)s.d_rmsq, (void *)s.d_boff, (void *)s.d_keys})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)s.h_ref, s.h_k, (void *)s.h_rmsq, (void *)s.h_boff, (void *)s.h_keys})
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : {s.ev_in, s.ev_free})
        if (e) (void)hipEventDestroy(e);
    s = pbg::StreamSlot{};
}

// positions and keys a slot must hold; grows (after its last use has finished) when short
int ensure_slot(pbg_ctx *c, pbg::StreamSlot &s, uint32_t chunk, size_t keys) {
    const int n = c->dp.n, kb = c->dp.k16 ? 2 : 1;
    if (!s.ev_in) {
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&s.ev_free, hipEventDisableTiming));
    }
    keys = std::max<size_t>(keys, 64);   // a chunk without keys still hands the kernels a keys pointer
    const bool need_pos = s.pos_cap < chunk;
    const bool need_keys = s.keys_cap < keys;
    if (!need_pos && !need_keys) return PBG_OK;
    if (s.used) {   // the slot's copies and call are done before its buffers go
        HIPCHK(c, hipEventSynchronize(s.ev_free));
        HIPCHK(c, hipEventSynchronize(s.ev_in));
    }
    const size_t nb = chunk / pbg::kSiteBlock + 2;
    if (need_pos) {
        for (void *p : {(void *)s.d_ref, s.d_k, (void *)s.d_rmsq, (void *)s.d_boff})
            if (p) HIPCHK(c, hipFree(p));
        for (void *p : {(void *)s.h_ref, s.h_k, (void *)s.h_rmsq, (void *)s.h_boff})
            if (p) HIPCHK(c, hipHostFree(p));
        s.d_ref = nullptr, s.d_k = nullptr, s.d_rmsq = nullptr, s.d_boff = nullptr;
        s.h_ref = nullptr, s.h_k = nullptr, s.h_rmsq = nullptr, s.h_boff = nullptr;
        HIPCHK(c, hipMalloc((void **)&s.d_ref, (size_t)chunk + 16));
        HIPCHK(c, hipMalloc(&s.d_k, (size_t)chunk * n * kb + 16));
        HIPCHK(c, hipMalloc((void **)&s.d_rmsq, (size_t)chunk * n * 4 + 16));
        HIPCHK(c, hipMalloc((void **)&s.d_boff, nb * 8));
        HIPCHK(c, hipHostMalloc((void **)&s.h_ref, (size_t)chunk + 16, hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc(&s.h_k, (size_t)chunk * n * kb + 16, hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc((void **)&s.h_rmsq, (size_t)chunk * n * 4 + 16, hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc((void **)&s.h_boff, nb * 8, hipHostMallocDefault));
        s.pos_cap = chunk;
    }
    if (need_keys) {
        if (s.d_keys) HIPCHK(c, hipFree(s.d_keys));
        if (s.h_keys) HIPCHK(c, hipHostFree(s.h_keys));
        s.d_keys = nullptr;
        s.h_keys = nullptr;
        const size_t cap = (keys + keys / 4 + 64) & ~(size_t)7;   // + 25 %: chunks vary in depth
        HIPCHK(c, hipMalloc((void **)&s.d_keys, cap * 2 + 16));
        HIPCHK(c, hipHostMalloc((void **)&s.h_keys, cap * 2 + 16, hipHostMallocDefault));
        s.keys_cap = s.h_keys_cap = cap;
    }
    return PBG_OK;
}

// a pair of timing events from the context's pool
int ev_pair(pbg_stream *st, int kind, hipEvent_t &a, hipEvent_t &b) {
    pbg_ctx *c = st->c;
    auto &ev = c->sb.ev;
    if (st->ev_kind.size() == ev.size()) {
        hipEvent_t x, y;
        HIPCHK(c, hipEventCreate(&x));
        HIPCHK(c, hipEventCreate(&y));
        ev.emplace_back(x, y);
    }
    a = ev[st->ev_kind.size()].first;
    b = ev[st->ev_kind.size()].second;
    st->ev_kind.push_back(kind);
    return PBG_OK;
}

// main_<cmd>'s windows (pop_nucdiv.cpp:47-72): [beg + cw*w, beg + (cw+1)*w - 1) for
// cw < ((end-beg)-1)/w (the last base of each window and the trailing partial window are
// dropped), or the whole region without -w
std::vector<std::pair<int32_t, int32_t>> command_windows(const pbg_cmd &cmd) {
    std::vector<std::pair<int32_t, int32_t>> win;
    if (cmd.windowed) {
        const int64_t w = cmd.win_size;
        const int64_t nw = ((int64_t)(cmd.end - cmd.beg) - 1) / w;
        for (int64_t cw = 0; cw < nw; ++cw)
            win.emplace_back((int32_t)(cmd.beg + cw * w), (int32_t)((cw + 1) * w + (cmd.beg - 1)));
    } else {
        win.emplace_back(cmd.beg, cmd.end);
    }
    return win;
}

// a device copy of a command's row-range window list, kept by content in the context (the
// window-statistics plan cache is keyed by the device pointer, which therefore stays valid)
int window_list(pbg_ctx *c, const pbg_cmd &cmd, int64_t dpos0, uint32_t dsites,
                const std::vector<std::pair<int32_t, int32_t>> &win, const pbg_window **out) {
    auto &wl = c->sb.wins;
    for (size_t i = 0; i < wl.size(); ++i) {
        const pbg::WinList &x = wl[i];
        if (x.windowed == cmd.windowed && x.win_size == (cmd.windowed ? cmd.win_size : 0) && x.beg == cmd.beg &&
            x.end == cmd.end && x.dpos0 == (int32_t)dpos0 && x.dsites == dsites && x.n_win == (uint32_t)win.size()) {
            *out = x.d;
            return PBG_OK;
        }
    }
    std::vector<pbg_window> rw(win.size());
    for (size_t i = 0; i < win.size(); ++i) {   // clipped to the rows (positions outside have no callback)
        const int64_t a = std::min<int64_t>(std::max<int64_t>(win[i].first, dpos0), dpos0 + dsites);
        const int64_t b = std::min<int64_t>(std::max<int64_t>(win[i].second, a), dpos0 + dsites);
        rw[i].beg = (int32_t)(a - dpos0);
        rw[i].end = (int32_t)(b - dpos0);
    }
    if (wl.size() >= 8) {   // evict the oldest and every plan made on it
        HIPCHK(c, hipDeviceSynchronize());
        const void *d = wl.front().d;
        c->plans.erase(std::remove_if(c->plans.begin(), c->plans.end(), [&](const pbg_ctx::Plan &p) { return p.wins == d; }),
                       c->plans.end());
        HIPCHK(c, hipFree(wl.front().d));
        wl.erase(wl.begin());
    }
    pbg::WinList x{cmd.windowed, cmd.beg, cmd.end, (int32_t)dpos0, cmd.windowed ? cmd.win_size : 0, dsites,
                   (uint32_t)win.size(), nullptr};
    HIPCHK(c, hipMalloc((void **)&x.d, std::max<size_t>(1, rw.size()) * sizeof(pbg_window)));
    if (!rw.empty()) HIPCHK(c, hipMemcpy(x.d, rw.data(), rw.size() * sizeof(pbg_window), hipMemcpyHostToDevice));
    wl.push_back(x);
    *out = x.d;
    return PBG_OK;
}

// print_<cmd> of one command over the region's rows (device; dsites rows from contig position
// dpos0), its consensus words (snp -o 0) and the region's reference bytes
int format_command(pbg_ctx *c, const pbg_cmd *cmd, const void *d_rows, uint32_t dsites, int64_t dpos0,
                   const uint64_t *d_cb, const uint8_t *href, hipStream_t s, std::string &text) {
    const int n = c->dp.n, np = c->dp.npops;
    const int rb = row_bytes_of(c);
    const auto win = command_windows(*cmd);
    if (cmd->cmd == PBG_CMD_SNP) {
        // print_snp per window (pop_snp.cpp:218-317): segregating positions in order, as
        // print_popbam_snp (-o 0), print_sweep (-o 1) or print_ms (-o 2, header first)
        if (cmd->output < 0 || cmd->output > 2) return fail(c, PBG_E_ARG, "snp output format must be 0, 1 or 2");
        const bool words = cmd->output == 0;
        std::vector<unsigned char> rows((size_t)dsites * rb);
        std::vector<uint64_t> cb(words ? (size_t)dsites * n : 0);
        if (dsites) {
            HIPCHK(c, hipMemcpyAsync(rows.data(), d_rows, rows.size(), hipMemcpyDeviceToHost, s));
            if (words) HIPCHK(c, hipMemcpyAsync(cb.data(), d_cb, cb.size() * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
        }
        using pbg::mask128;
        const mask128 tmask = ((mask128)1 << n) - 1;   // n <= 126
        std::vector<mask128> pmask(np);
        for (int i = 0; i < np; ++i) pmask[i] = ((mask128)c->dp.pop_mask_hi[i] << 64) | c->dp.pop_mask[i];
        // print_ms prints its header in the window loop at cw == 0 (pop_snp.cpp:114-115): not at
        // all without windows; a block of a longer run passes the run's count or suppresses it
        if (cmd->output == 2 && cmd->ms_windows >= 0 && !win.empty())
            pbg::format_ms_header(text, n, np, c->params.pop_n, cmd->ms_windows > 0 ? (long)cmd->ms_windows : (long)win.size());
        std::vector<int32_t> wpos;
        std::vector<mask128> wtypes;
        for (auto &x : win) {
            wpos.clear();
            wtypes.clear();
            for (int64_t p = std::max<int64_t>(x.first, dpos0); p < std::min<int64_t>(x.second, dpos0 + dsites); ++p) {
                const size_t i = (size_t)(p - dpos0);
                const unsigned char *r = rows.data() + i * rb;
                if (!((r[rb - 1] >> 7) & 1)) continue;   // not segregating
                mask128 types = 0;
                for (int b = 0; b < rb; ++b) types |= (mask128)r[b] << (8 * b);
                types &= tmask;
                if (cmd->output == 0)
                    pbg::format_snp_site(text, *cmd, n, (int32_t)p, href[i] & 0x7f, cb.data() + i * n);
                else if (cmd->output == 1)
                    pbg::format_sweep_site(text, *cmd, np, pmask.data(), c->params.flag, (int32_t)p, types);
                wpos.push_back((int32_t)p);
                wtypes.push_back(types);
            }
            if (cmd->output == 2) pbg::format_ms_window(text, n, c->params.flag, cmd->outidx, x.first, x.second, wpos, wtypes);
        }
        return PBG_OK;
    }
    uint32_t stats = 0;
    switch (cmd->cmd) {
        case PBG_CMD_NUCDIV: stats = PBG_S_NUCDIV; break;
        case PBG_CMD_SFS: stats = PBG_S_SFS; break;
        case PBG_CMD_LD: stats = cmd->output == 1 ? PBG_S_OMEGA : cmd->output == 2 ? PBG_S_WALL : PBG_S_ZNS; break;
        case PBG_CMD_DIVERGE: stats = cmd->output == 1 ? PBG_S_DIV_POP : PBG_S_DIV_IND; break;
        case PBG_CMD_HAPLO:
            stats = cmd->output == 1 ? PBG_S_HAP_EHHS : cmd->output == 2 ? PBG_S_HAP_DXY : PBG_S_HAP_K;
            break;
        case PBG_CMD_TREE:
            // join_tree's last cycle needs three clusters (ntaxa = n + 1 >= 3)
            if (n < 2) return fail(c, PBG_E_ARG, "tree needs at least two samples");
            stats = PBG_S_TREE;
            break;
        default: return fail(c, PBG_E_ARG, "unsupported subcommand");
    }
    const uint32_t nw = (uint32_t)win.size();
    if (nw == 0) return PBG_OK;
    const pbg_window *d_win = nullptr;
    int rc = window_list(c, *cmd, dpos0, dsites, win, &d_win);
    if (rc) return rc;
    // outputs: one device block, carved per field (reused by the next command)
    const int npairs = std::max(1, np * (np - 1));
    const size_t szw = nw, szp = (size_t)nw * np, szq = (size_t)nw * npairs, szn = (size_t)nw * n;
    const size_t szt = stats == PBG_S_TREE ? (size_t)nw * (n + 1) * (n + 1) : 1;
    const bool theta = stats == PBG_S_SFS && (cmd->output & 1);   // sfs --theta
    const size_t szb = theta ? szp * (size_t)c->dp.sfs_stride : 1;
    const size_t n_d1 = std::max(szq, std::max(szp, szn)), n_d2 = std::max(szq, szp), n_d3 = szp;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b_ns = al(szw * 4), b_seg = al(szw * 4), b_d1 = al(n_d1 * 8), b_d2 = al(n_d2 * 8), b_d3 = al(n_d3 * 8),
                 b_i1 = al(szp * 4), b_i2 = al(szp * 4), b_i3 = al(szq * 4), b_td = al(szt * 4), b_bins = al(szb * 4);
    const size_t need = b_ns + b_seg + b_d1 + b_d2 + b_d3 + b_i1 + b_i2 + b_i3 + b_td + b_bins;
    if (c->sb.out_cap < need) {
        if (c->sb.d_out) HIPCHK(c, hipFree(c->sb.d_out));
        c->sb.d_out = nullptr;
        HIPCHK(c, hipMalloc(&c->sb.d_out, need));
        c->sb.out_cap = need;
    }
    char *o = (char *)c->sb.d_out;
    int32_t *o_ns = (int32_t *)o;                o += b_ns;
    int32_t *o_seg = (int32_t *)o;               o += b_seg;
    double *d1 = (double *)o;                    o += b_d1;
    double *d2 = (double *)o;                    o += b_d2;
    double *d3 = (double *)o;                    o += b_d3;
    int32_t *i1 = (int32_t *)o;                  o += b_i1;
    int32_t *i2 = (int32_t *)o;                  o += b_i2;
    int32_t *i3 = (int32_t *)o;                  o += b_i3;
    int32_t *o_td = (int32_t *)o;                o += b_td;
    int32_t *o_bins = (int32_t *)o;
    pbg_window_out O{};
    O.num_sites = o_ns;
    O.segsites = o_seg;
    switch (stats) {
        case PBG_S_NUCDIV: O.pi = d1; O.dxy = d2; break;
        case PBG_S_SFS:
            O.td = d1; O.fwh = d2;
            if (theta) { O.seg_pop = i1; O.theta_w = d3; O.sfs_bins = o_bins; }
            break;
        case PBG_S_ZNS: case PBG_S_OMEGA: O.ld_snps = i1; O.ld_val = d1; break;
        case PBG_S_WALL: O.ld_snps = i1; O.ld_val = d1; O.ld_q = d2; break;
        case PBG_S_DIV_IND: O.div_ind = d1; break;
        case PBG_S_DIV_POP: O.div_fixed = i1; O.div_seg = i2; O.div_pop = d1; break;
        case PBG_S_HAP_K: O.nhaps = i1; O.hap_val = d1; break;
        case PBG_S_HAP_EHHS: O.hap_val = d1; break;
        case PBG_S_HAP_DXY: O.hap_val = d3; O.hap_dxy = d1; O.hap_min = i3; break;
        case PBG_S_TREE: O.tree_diff = o_td; break;
    }
    pbg_stat_opts so{stats, cmd->min_freq, cmd->outidx, cmd->jc};
    if ((rc = pbg_window_stats(c, d_rows, dsites, d_win, nw, &so, &O, s))) return rc;
    if ((rc = pbg_check(c, s))) return rc;
    std::vector<int32_t> h_ns(szw), h_seg(szw), h_i1(szp), h_i2(szp), h_i3(szq), h_td(szt), h_bins(szb);
    std::vector<double> h_d1(n_d1), h_d2(n_d2), h_d3(n_d3);
    auto d2h = [&](void *dst, const void *src, size_t bytes) { return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s); };
    HIPCHK(c, d2h(h_ns.data(), o_ns, szw * 4));
    HIPCHK(c, d2h(h_seg.data(), o_seg, szw * 4));
    HIPCHK(c, d2h(h_i1.data(), i1, szp * 4));
    HIPCHK(c, d2h(h_i2.data(), i2, szp * 4));
    HIPCHK(c, d2h(h_i3.data(), i3, szq * 4));
    if (stats == PBG_S_TREE) HIPCHK(c, d2h(h_td.data(), o_td, szt * 4));
    if (theta) HIPCHK(c, d2h(h_bins.data(), o_bins, szb * 4));
    HIPCHK(c, d2h(h_d1.data(), d1, n_d1 * 8));
    HIPCHK(c, d2h(h_d2.data(), d2, n_d2 * 8));
    HIPCHK(c, d2h(h_d3.data(), d3, n_d3 * 8));
    HIPCHK(c, hipStreamSynchronize(s));
    pbg::WindowHost wh;
    auto slice = [](const auto &v, size_t off, size_t cnt) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        return std::vector<T>(v.begin() + off, v.begin() + off + cnt);
    };
    for (uint32_t i = 0; i < nw; ++i) {
        wh.beg = win[i].first;
        wh.end = win[i].second;
        wh.num_sites = h_ns[i];
        wh.segsites = h_seg[i];
        switch (stats) {
            case PBG_S_NUCDIV: wh.pi = slice(h_d1, i * np, np); wh.dxy = slice(h_d2, (size_t)i * npairs, npairs); break;
            case PBG_S_SFS:
                wh.td = slice(h_d1, i * np, np); wh.fwh = slice(h_d2, i * np, np);
                if (theta) {
                    wh.seg_pop = slice(h_i1, i * np, np); wh.theta_w = slice(h_d3, i * np, np);
                    wh.sfs_bins.assign(np, {});
                    for (int p = 0; p < np; ++p)
                        wh.sfs_bins[p] = slice(h_bins, ((size_t)i * np + p) * c->dp.sfs_stride, (size_t)c->dp.pop_n[p] + 1);
                }
                break;
            case PBG_S_ZNS: case PBG_S_OMEGA:
                wh.ld_snps = slice(h_i1, i * np, np); wh.ld_val = slice(h_d1, i * np, np); break;
            case PBG_S_WALL:
                wh.ld_snps = slice(h_i1, i * np, np); wh.ld_val = slice(h_d1, i * np, np);
                wh.ld_q = slice(h_d2, i * np, np); break;
            case PBG_S_DIV_IND: wh.div_ind = slice(h_d1, (size_t)i * n, n); break;
            case PBG_S_DIV_POP:
                wh.div_fixed = slice(h_i1, i * np, np); wh.div_seg = slice(h_i2, i * np, np);
                wh.div_pop = slice(h_d1, i * np, np); break;
            case PBG_S_HAP_K: wh.nhaps = slice(h_i1, i * np, np); wh.hap_val = slice(h_d1, i * np, np); break;
            case PBG_S_HAP_EHHS: wh.hap_val = slice(h_d1, i * np, np); break;
            case PBG_S_HAP_DXY:
                wh.hap_val = slice(h_d3, i * np, np); wh.hap_dxy = slice(h_d1, (size_t)i * npairs, npairs);
                wh.hap_min = slice(h_i3, (size_t)i * npairs, npairs); break;
            case PBG_S_TREE: wh.tree_diff = slice(h_td, (size_t)i * (n + 1) * (n + 1), (size_t)(n + 1) * (n + 1)); break;
        }
        pbg::format_window(text, *cmd, n, np, c->dp.flag, wh);
    }
    return PBG_OK;
}

}  // namespace

void pbg::stream_bufs_free(pbg_ctx *c) {
    pbg::StreamBufs &b = c->sb;
    for (auto &s : b.slot) free_slot(s);
    for (void *p : {b.d_rows, (void *)b.d_cb, b.d_out})
        if (p) (void)hipFree(p);
    for (auto &w : b.wins)
        if (w.d) (void)hipFree(w.d);
    for (auto &e : b.ev) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (hipStream_t s : {b.copy, b.comp})
        if (s) (void)hipStreamDestroy(s);
    b = pbg::StreamBufs{};
}

extern "C" {

int pbg_stream_open(pbg_ctx *c, const pbg_cmd *cmds, uint32_t n_cmd, int32_t pos0, uint32_t n_sites,
                    uint32_t chunk_sites, pbg_stream **out) {
    if (!c || !out || (n_cmd && !cmds)) return fail(c, PBG_E_ARG, "null argument");
    *out = nullptr;
    for (uint32_t i = 0; i < n_cmd; ++i)
        if (cmds[i].windowed && cmds[i].win_size <= 0) return fail(c, PBG_E_ARG, "window size must be positive");
    HIPCHK(c, hipSetDevice(c->device));
    pbg::StreamBufs &b = c->sb;
    if (!b.copy) HIPCHK(c, hipStreamCreateWithFlags(&b.copy, hipStreamNonBlocking));
    if (!b.comp) HIPCHK(c, hipStreamCreateWithFlags(&b.comp, hipStreamNonBlocking));
    const int n = c->dp.n, kb = c->dp.k16 ? 2 : 1, rb = c->row_bytes;
    pbg_stream *st = new pbg_stream();
    st->c = c;
    st->cmds.assign(cmds, cmds + n_cmd);
    st->pos0 = pos0;
    st->n_sites = n_sites;
    for (uint32_t i = 0; i < n_cmd; ++i) st->words |= cmds[i].cmd == PBG_CMD_SNP && cmds[i].output == 0;
    // chunk: about 256 MB of (k, sum mapQ^2, keys at depth ~10) per slot, a multiple of 64
    uint64_t ch = chunk_sites ? chunk_sites : (uint64_t)(256u << 20) / ((uint64_t)n * (kb + 4 + 20) + 1);
    ch = std::max<uint64_t>(pbg::kSiteBlock, std::min<uint64_t>(ch, std::max<uint32_t>(n_sites, 1)));
    st->chunk = (uint32_t)((ch + pbg::kSiteBlock - 1) / pbg::kSiteBlock * pbg::kSiteBlock);
    const size_t rows_bytes = ((size_t)n_sites * rb + 255) & ~(size_t)255;
    if (b.rows_cap < rows_bytes || !b.d_rows) {
        if (b.d_rows) {
            HIPCHK(c, hipStreamSynchronize(b.comp));
            HIPCHK(c, hipFree(b.d_rows));
        }
        b.d_rows = nullptr;
        HIPCHK(c, hipMalloc(&b.d_rows, std::max<size_t>(rows_bytes, 256)));
        b.rows_cap = std::max<size_t>(rows_bytes, 256);
    }
    if (n_sites) HIPCHK(c, hipMemsetAsync(b.d_rows, 0, rows_bytes, b.comp));   // unpushed positions: uncounted
    if (st->words) {
        const size_t cbb = (size_t)n_sites * n * 8;
        if (b.cb_cap < cbb) {
            if (b.d_cb) {
                HIPCHK(c, hipStreamSynchronize(b.comp));
                HIPCHK(c, hipFree(b.d_cb));
            }
            b.d_cb = nullptr;
            HIPCHK(c, hipMalloc((void **)&b.d_cb, cbb + 16));
            b.cb_cap = cbb;
        }
        st->href.assign(n_sites, 0x80);
    }
    *out = st;
    return PBG_OK;
}

}  // extern "C"

namespace {

int stream_push(pbg_stream *st, const pbg_pileup *pc, bool compact) {
    pbg_ctx *c = st->c;
    if (st->finished) return fail(c, PBG_E_ARG, "stream already finished");
    if (compact && st->words) return fail(c, PBG_E_ARG, "compact pieces carry no keys for reference-only tasks: no consensus words (snp -o 0)");
    // a compact piece flags a task in bit 31 of its sum mapQ^2, which no unflagged task may reach:
    // at most 255^2 per read, so max_depth <= 33025
    if (compact && c->dp.max_depth > 33025) return fail(c, PBG_E_ARG, "compact pieces need max_depth <= 33025");
    if (pc->n_sites == 0) return PBG_OK;
    if (!pc->ref || !pc->k || !pc->rmsq || !pc->keys) return fail(c, PBG_E_ARG, "null pileup array");
    if ((int64_t)pc->pos0 != (int64_t)st->pos0 + st->pushed) return fail(c, PBG_E_ARG, "pieces must be pushed in position order");
    if ((uint64_t)st->pushed + pc->n_sites > st->n_sites) return fail(c, PBG_E_RANGE, "piece beyond the stream's region");
    if (st->pushed + pc->n_sites < st->n_sites && (pc->n_sites % pbg::kSiteBlock))
        return fail(c, PBG_E_ARG, "every piece but the last must hold a multiple of 64 positions");
    HIPCHK(c, hipSetDevice(c->device));
    pbg::StreamBufs &b = c->sb;
    const int n = c->dp.n, kb = c->dp.k16 ? 2 : 1, rb = c->row_bytes;
    const uint32_t L = pc->n_sites, nblk = (L + pbg::kSiteBlock - 1) / pbg::kSiteBlock;
    std::vector<uint64_t> own;
    const uint64_t *boff = pc->block_off;
    if (!boff) {   // derived from k[] (the callback's per-sample key counts)
        own.assign(nblk + 1, 0);
        uint64_t run = 0;
        for (uint32_t bk = 0; bk < nblk; ++bk) {
            own[bk] = run;
            const size_t t1 = (size_t)std::min<uint32_t>(L, (bk + 1) * pbg::kSiteBlock) * n;
            for (size_t i = (size_t)bk * pbg::kSiteBlock * n; i < t1; ++i)
                if (!compact || !(pc->rmsq[i] >> 31))   // a flagged task's keys are not in the piece
                    run += kb == 1 ? ((const uint8_t *)pc->k)[i] : ((const uint16_t *)pc->k)[i];
        }
        own[nblk] = run;
        boff = own.data();
    }
    // pinned caller buffers are copied straight by the DMA engine (asynchronously: they must stay
    // unchanged until pbg_stream_finish); pageable ones through the slot's pinned staging
    const bool pinned = is_pinned(pc->ref) && is_pinned(pc->k) && is_pinned(pc->rmsq) && is_pinned(pc->keys);
    ++st->prof.pieces;
    for (uint32_t p0 = 0; p0 < L; p0 += st->chunk) {
        const uint32_t p1 = std::min(L, p0 + st->chunk), cl = p1 - p0;
        const uint32_t b0 = p0 / pbg::kSiteBlock, b1 = (p1 + pbg::kSiteBlock - 1) / pbg::kSiteBlock;
        const uint64_t ka = boff[b0] & ~(uint64_t)7, kz = boff[b1];
        if (kz < boff[b0]) return st->rc = fail(c, PBG_E_BATCH, "block_off decreases");
        const size_t nk = (size_t)(kz - ka);
        pbg::StreamSlot &s = b.slot[st->cur];
        st->cur ^= 1;
        const auto tw = Clock::now();
        // a slot grows to the largest chunk it has held: pieces smaller than the stream's chunk (the
        // feeder's 64 k-position pieces) pin and allocate only what they need
        int rc = ensure_slot(c, s, (cl + pbg::kSiteBlock - 1) / pbg::kSiteBlock * pbg::kSiteBlock, nk);
        if (rc) return st->rc = rc;
        if (s.used) HIPCHK(c, hipEventSynchronize(s.ev_in));   // its staging is free again
        st->prof.ms_wait += ms_since(tw);
        const size_t t0 = (size_t)p0 * n;
        const void *src_ref = pc->ref + p0, *src_k = (const char *)pc->k + t0 * kb, *src_rq = pc->rmsq + t0,
                   *src_keys = pc->keys + ka;
        std::memcpy(s.h_boff, boff + b0, (size_t)(b1 - b0 + 1) * 8);
        if (!pinned) {
            const auto ts = Clock::now();
            par_copy({{s.h_ref, src_ref, cl}, {s.h_k, src_k, (size_t)cl * n * kb}, {s.h_rmsq, src_rq, (size_t)cl * n * 4},
                      {s.h_keys, src_keys, nk * 2}});
            st->prof.ms_stage += ms_since(ts);
            src_ref = s.h_ref, src_k = s.h_k, src_rq = s.h_rmsq, src_keys = s.h_keys;
        } else {
            ++st->prof.pinned_chunks;
        }
        hipEvent_t e0, e1;
        if ((rc = ev_pair(st, 0, e0, e1))) return st->rc = rc;
        if (s.used) HIPCHK(c, hipStreamWaitEvent(b.copy, s.ev_free, 0));   // its previous call is done
        HIPCHK(c, hipEventRecord(e0, b.copy));
        HIPCHK(c, hipMemcpyAsync(s.d_ref, src_ref, cl, hipMemcpyHostToDevice, b.copy));
        HIPCHK(c, hipMemcpyAsync(s.d_k, src_k, (size_t)cl * n * kb, hipMemcpyHostToDevice, b.copy));
        HIPCHK(c, hipMemcpyAsync(s.d_rmsq, src_rq, (size_t)cl * n * 4, hipMemcpyHostToDevice, b.copy));
        HIPCHK(c, hipMemcpyAsync(s.d_boff, s.h_boff, (size_t)(b1 - b0 + 1) * 8, hipMemcpyHostToDevice, b.copy));
        if (nk) HIPCHK(c, hipMemcpyAsync(s.d_keys, src_keys, nk * 2, hipMemcpyHostToDevice, b.copy));
        HIPCHK(c, hipEventRecord(e1, b.copy));
        HIPCHK(c, hipEventRecord(s.ev_in, b.copy));
        st->prof.h2d_bytes += (uint64_t)cl * (1 + (size_t)n * (kb + 4)) + (uint64_t)(b1 - b0 + 1) * 8 + nk * 2;
        HIPCHK(c, hipStreamWaitEvent(b.comp, s.ev_in, 0));
        // block_off keeps the piece's key offsets: the keys pointer is the slot shifted back to
        // the chunk's first (16-byte aligned) key (include/popbam_gpu.h allows it)
        const int64_t cpos = (int64_t)pc->pos0 + p0;
        const uint64_t roff = (uint64_t)(cpos - st->pos0);
        pbg_pileup dp{cl, (int32_t)cpos, s.d_ref, s.d_k, s.d_rmsq, s.d_boff, s.d_keys - ka};
        hipEvent_t c0, c1;
        if ((rc = ev_pair(st, 1, c0, c1))) return st->rc = rc;
        HIPCHK(c, hipEventRecord(c0, b.comp));
        c->scan_masked = masked_reference(pc->ref + p0, cl) ? 1 : 0;
        c->scan_compact = compact ? 1 : 0;
        c->cap_hint_keys = (int64_t)(boff[b1] - boff[b0]);
        rc = pbg_call_sites(c, &dp, (char *)b.d_rows + roff * rb, st->words ? b.d_cb + roff * n : nullptr, b.comp);
        c->scan_masked = 0;
        c->scan_compact = 0;
        c->cap_hint_keys = -1;
        if (rc) return st->rc = rc;
        HIPCHK(c, hipEventRecord(c1, b.comp));
        HIPCHK(c, hipEventRecord(s.ev_free, b.comp));
        s.used = true;
        ++st->prof.chunks;
    }
    if (st->words) std::memcpy(st->href.data() + st->pushed, pc->ref, L);
    st->pushed += L;
    return PBG_OK;
}

int stream_finish(pbg_stream *st) {
    pbg_ctx *c = st->c;
    const auto t0 = Clock::now();
    st->finished = true;
    if (st->pushed != st->n_sites) return st->rc = fail(c, PBG_E_RANGE, "the pushed pieces do not cover the stream's region");
    HIPCHK(c, hipSetDevice(c->device));
    pbg::StreamBufs &b = c->sb;
    int rc = pbg_check(c, b.comp);   // waits for every call; an inconsistent batch is an error here
    if (rc) return st->rc = rc;
    for (size_t i = 0; i < st->ev_kind.size(); ++i) {
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, b.ev[i].first, b.ev[i].second));
        (st->ev_kind[i] ? st->prof.ms_call : st->prof.ms_h2d) += ms;
    }
    // an all-empty region still needs one addressable row for the kernels' pointer
    st->text.assign(st->cmds.size(), std::string());
    for (size_t i = 0; i < st->cmds.size(); ++i) {
        rc = format_command(c, &st->cmds[i], b.d_rows, st->n_sites, st->pos0, st->words ? b.d_cb : nullptr,
                            st->href.data(), b.comp, st->text[i]);
        if (rc) return st->rc = rc;
    }
    st->prof.ms_finish = ms_since(t0);
    return PBG_OK;
}

}  // namespace

extern "C" {

// every failure of push / finish (argument, HIP, batch) is the stream's sticky error: a later
// push, finish or text of that stream returns it instead of a misleading order / coverage error
int pbg_stream_push(pbg_stream *st, const pbg_pileup *pc) {
    if (!st || !pc) return PBG_E_ARG;
    if (st->rc) return st->rc;
    const int rc = stream_push(st, pc, false);
    if (rc) st->rc = rc;
    return rc;
}

int pbg_stream_push_compact(pbg_stream *st, const pbg_pileup *pc) {
    if (!st || !pc) return PBG_E_ARG;
    if (st->rc) return st->rc;
    const int rc = stream_push(st, pc, true);
    if (rc) st->rc = rc;
    return rc;
}

int pbg_stream_finish(pbg_stream *st) {
    if (!st) return PBG_E_ARG;
    if (st->finished || st->rc) return st->rc;
    const int rc = stream_finish(st);
    if (rc) st->rc = rc;
    return rc;
}

long pbg_stream_text(pbg_stream *st, uint32_t i, char *out, size_t cap, size_t *needed) {
    if (!st || (!out && cap)) return PBG_E_ARG;
    pbg_ctx *c = st->c;
    if (!st->finished) return fail(c, PBG_E_ARG, "pbg_stream_finish first");
    if (st->rc) return st->rc;
    if (i >= st->text.size()) return fail(c, PBG_E_ARG, "command index out of range");
    const std::string &t = st->text[i];
    if (needed) *needed = t.size() + 1;
    if (t.size() + 1 > cap) return fail(c, PBG_E_RANGE, "output buffer too small");
    std::memcpy(out, t.c_str(), t.size() + 1);
    return (long)t.size();
}

int pbg_stream_rows(const pbg_stream *st, void *dst, size_t cap) {
    if (!st || (!dst && cap)) return PBG_E_ARG;
    pbg_ctx *c = st->c;
    const size_t bytes = (size_t)st->n_sites * c->row_bytes;
    if (cap < bytes) return fail(c, PBG_E_RANGE, "rows buffer too small");
    if (!bytes) return PBG_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, c->sb.d_rows, bytes, hipMemcpyDefault, c->sb.comp));
    HIPCHK(c, hipStreamSynchronize(c->sb.comp));
    return PBG_OK;
}

int pbg_stream_profile(const pbg_stream *st, pbg_stream_prof *p) {
    if (!st || !p) return PBG_E_ARG;
    *p = st->prof;
    return PBG_OK;
}

const char *pbg_stream_error(const pbg_stream *st) {
    if (!st) return "null stream";
    if (!st->rc) return "";
    return pbg_last_error(st->c);
}

void pbg_stream_close(pbg_stream *st) {
    if (!st) return;
    if (st->c && st->c->sb.comp) {
        (void)hipSetDevice(st->c->device);
        (void)hipStreamSynchronize(st->c->sb.comp);   // no call may still read a slot / write the rows
        (void)hipStreamSynchronize(st->c->sb.copy);
        // a stream that failed or never finished may leave kernel flags behind (its pbg_check never
        // ran): clear them, so the context's next run does not report this one's batch
        if ((st->rc || !st->finished) && st->c->d_err) (void)hipMemset(st->c->d_err, 0, sizeof(int));
    }
    delete st;
}

long pbg_run(pbg_ctx *c, const pbg_cmd *cmd, const pbg_pileup *hp, char *out, size_t cap, size_t *needed) {
    if (!c || !cmd || !hp || (!out && cap)) return fail(c, PBG_E_ARG, "null argument");
    if (hp->n_sites && (!hp->ref || !hp->k || !hp->rmsq || !hp->keys)) return fail(c, PBG_E_ARG, "null pileup array");
    if (cmd->windowed && cmd->win_size <= 0) return fail(c, PBG_E_ARG, "window size must be positive");
    c->text.clear();
    const int n = c->dp.n, kb = c->dp.k16 ? 2 : 1;
    // the 64-position blocks of the batch the command's windows touch
    const auto win = command_windows(*cmd);
    const int64_t pos0 = hp->pos0, pend = (int64_t)hp->pos0 + hp->n_sites;
    int64_t lo = pend, hi = pos0;
    for (auto &x : win) {
        const int64_t a = std::max<int64_t>(x.first, pos0), e = std::min<int64_t>(x.second, pend);
        if (a < e) {
            lo = std::min(lo, a);
            hi = std::max(hi, e);
        }
    }
    uint32_t blo = 0, dsites = 0;
    if (lo < hi) {
        blo = (uint32_t)((lo - pos0) / pbg::kSiteBlock);
        const uint32_t bhi = (uint32_t)((hi - pos0 + pbg::kSiteBlock - 1) / pbg::kSiteBlock);
        dsites = std::min<uint32_t>(hp->n_sites, bhi * pbg::kSiteBlock) - blo * pbg::kSiteBlock;
    }
    const int64_t dpos0 = pos0 + (int64_t)blo * pbg::kSiteBlock;
    std::vector<uint64_t> own;
    const uint64_t *hboff = hp->block_off;
    if (dsites && !hboff) {   // the piece's block offsets (into hp->keys), from k[]
        const uint32_t nb = (dsites + pbg::kSiteBlock - 1) / pbg::kSiteBlock;
        own.assign(blo + nb + 1, 0);
        uint64_t run = 0;
        const size_t tend = (size_t)(blo * pbg::kSiteBlock + dsites) * n;
        for (size_t i = 0; i < (size_t)blo * pbg::kSiteBlock * n; ++i)
            run += kb == 1 ? ((const uint8_t *)hp->k)[i] : ((const uint16_t *)hp->k)[i];
        for (uint32_t bk = blo; bk < blo + nb; ++bk) {
            own[bk] = run;
            const size_t t1 = std::min(tend, (size_t)(bk + 1) * pbg::kSiteBlock * n);
            for (size_t i = (size_t)bk * pbg::kSiteBlock * n; i < t1; ++i)
                run += kb == 1 ? ((const uint8_t *)hp->k)[i] : ((const uint16_t *)hp->k)[i];
        }
        own[blo + nb] = run;
        hboff = own.data();
    }
    pbg_stream *st = nullptr;
    int rc = pbg_stream_open(c, cmd, 1, (int32_t)dpos0, dsites, 0, &st);
    if (rc) return rc;
    if (dsites) {
        const size_t t0 = (size_t)blo * pbg::kSiteBlock * n;
        pbg_pileup piece{dsites, (int32_t)dpos0, hp->ref + (size_t)blo * pbg::kSiteBlock, (const char *)hp->k + t0 * kb,
                         hp->rmsq + t0, hboff + blo, hp->keys};
        rc = pbg_stream_push(st, &piece);
    }
    if (!rc) rc = pbg_stream_finish(st);
    if (rc) {
        pbg_stream_close(st);
        return rc;
    }
    std::string text;
    text.swap(st->text[0]);
    pbg_stream_close(st);
    if (needed) *needed = text.size() + 1;
    if (text.size() + 1 > cap) {
        c->text.swap(text);   // kept for pbg_take_text
        return fail(c, PBG_E_RANGE, "output buffer too small");
    }
    std::memcpy(out, text.c_str(), text.size() + 1);
    return (long)text.size();
}

long pbg_take_text(pbg_ctx *c, char *out, size_t cap) {
    if (!c || (!out && cap)) return fail(c, PBG_E_ARG, "null argument");
    if (c->text.size() + 1 > cap) return fail(c, PBG_E_RANGE, "output buffer too small");
    std::memcpy(out, c->text.c_str(), c->text.size() + 1);
    const long len = (long)c->text.size();
    std::string().swap(c->text);
    return len;
}

}  // extern "C"
