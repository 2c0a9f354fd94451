// pbg_ctx.h -- the context behind the C-ABI handle (internal to libpopbam_gpu.so).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "pbg_common.h"
#include "pbg_host.h"

namespace pbg {

// One device slot of a streamed run (pbg_stream_push): a chunk of the pileup batch in HBM, and
// its pinned host staging (used when the caller's buffers are pageable).
struct StreamSlot {
    uint8_t *d_ref = nullptr;
    void *d_k = nullptr;
    uint32_t *d_rmsq = nullptr;
    uint64_t *d_boff = nullptr;
    uint16_t *d_keys = nullptr;
    uint32_t pos_cap = 0;                // positions
    size_t keys_cap = 0;                 // keys
    uint8_t *h_ref = nullptr;            // pinned staging
    void *h_k = nullptr;
    uint32_t *h_rmsq = nullptr;
    uint64_t *h_boff = nullptr;
    uint16_t *h_keys = nullptr;
    size_t h_keys_cap = 0;
    hipEvent_t ev_in = nullptr;          // its H2D copies done (copy stream)
    hipEvent_t ev_free = nullptr;        // the call reading it done (compute stream)
    bool used = false;
};
struct WinList {                         // a device window list, kept by content
    int32_t windowed, beg, end, dpos0;
    int64_t win_size;
    uint32_t dsites, n_win;
    pbg_window *d = nullptr;
};
struct StreamBufs {
    hipStream_t copy = nullptr, comp = nullptr;
    StreamSlot slot[2];
    void *d_rows = nullptr;
    size_t rows_cap = 0;
    uint64_t *d_cb = nullptr;
    size_t cb_cap = 0;
    void *d_out = nullptr;               // window outputs of one command
    size_t out_cap = 0;
    std::vector<WinList> wins;           // most recent last
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;   // profiling pairs
};

}  // namespace pbg

struct pbg_ctx {
    int device = 0;
    int n_cu = 256;   // the device's CU count (persistent queue-kernel grid)
    pbg_params params{};
    pbg::DevParams dp{};
    pbg::DevTables dt{};
    int row_bytes = 8;
    double *d_fk = nullptr, *d_beta = nullptr, *d_lhet = nullptr, *d_sfs = nullptr, *d_r2 = nullptr;
    double *d_fbeta = nullptr;
    double *d_lb = nullptr;
    double *d_oe = nullptr;
    void *d_scantab = nullptr;   // pbg::ScanTab (call_scan_kernel's LDS image)
    int *d_err = nullptr;
    int scan_masked = 0;   // the next pbg_call_sites' Batch::masked (set by pbg_stream_push from the host reference)
    int scan_compact = 0;  // the next pbg_call_sites' Batch::compact (set by pbg_stream_push_compact)
    std::string err;
    // per-pileup LDS staging capacity (keyed by block_off pointer and size), so repeated
    // calls on the same resident batch do not synchronise
    const void *cap_key = nullptr;
    uint32_t cap_sites = 0, cap_val = 0;
    int64_t cap_hint_keys = -1;   // the next pbg_call_sites' key count when the caller knows it on the
                                  // host (pbg_stream_push): no device read, no synchronisation
    // window lists already validated (device pointer, size, rows, statistics), most recent last
    struct Plan {
        const void *wins;
        uint32_t n_win, n_rows, stats;
        uint64_t zstride;   // ZnS list words per window at fixed places (0: pool)
        int segcap;         // segregating rows per window kept in LDS (WinLds::segcap)
    };
    std::vector<Plan> plans;
    uint64_t *d_ws = nullptr, *d_wsoff = nullptr, *d_zns = nullptr;
    size_t zns_cap = 0;   // bytes of d_zns
    size_t ws_cap = 0, wsoff_cap = 0, segcnt_cap = 0;
    int32_t *d_segcnt = nullptr;
    // samples deeper than the register sort width (call kernel): queues + parked info bytes
    pbg::DeepBufs deep{};
    size_t deep_sites_cap = 0, deep_info_cap = 0;
    // pbg_set_kernel_timing: HIP events around the dominant call kernel of every call, and
    // around the whole call
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev, evc;
    size_t ev_used = 0;
    // pbg_synth_pileup: block-total scan scratch; read-template tables per seed (built once,
    // never rebuilt while a generator launch on another stream may read them)
    uint64_t *d_synth = nullptr;
    size_t synth_cap = 0;
    std::vector<std::pair<uint64_t, uint16_t *>> tmpl;
    // pbg_run text kept when the caller's buffer was too small (pbg_take_text)
    std::string text;
    // streamed runs (stream.cpp): device slots, pinned staging, streams and window lists kept
    // for the next pbg_stream_open / pbg_run on this context
    pbg::StreamBufs sb;
};

namespace pbg {
int ctx_fail(pbg_ctx *c, int code, const std::string &msg);
void stream_bufs_free(pbg_ctx *c);
}  // namespace pbg

#define PBG_HIPCHK(ctx, expr)                                                                      \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return ::pbg::ctx_fail((ctx), PBG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)
