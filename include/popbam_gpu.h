/* popbam_gpu.h -- C-ABI of the MI355X-native POPBAM hot path (libpopbam_gpu.so).
 *
 * Drop-in boundary.  The reference drives its hot path through the pileup callback
 *     int (*bam_pileup_f)(uint32_t tid, uint32_t pos, int n, const bam_pileup1_t *pl, void *data)
 * (bam.h:554), registered per window with bam_plbuf_init(make_<cmd>, &t)
 * (bam_pileup.c:505-540) and implemented by make_nucdiv / make_sfs / make_ld / make_diverge /
 * make_haplo / make_snp (e.g. pop_nucdiv.cpp:136-204), each of which runs
 * popbamData::call_base (popbam.cpp:186-313) + clean_heterozygotes / segbase / qfilter
 * (pop_utils.cpp:102-201) per position and then calc_<stat> / print_<stat> per window.
 *
 * This library replaces everything after call_base's per-read loop:
 *   - the host side of the callback (reference popbam.cpp:220-287: skip is_del /
 *     is_refskip / BAM_FUNMAP, RG -> sample, keep the first max_depth reads per sample, then
 *     per read the baseQ / mapQ / N filters and the key qq<<5 | strand<<4 | base, plus the
 *     sum of mapQ^2) fills a pileup batch (pbg_pileup) with exactly the bytes SURVEY 8(d)
 *     counts: a u16 key per kept read, per (position, sample) the key count k (u8) and
 *     sum mapQ^2 (u32), per position the reference byte (libpopbam_feed.so does this);
 *   - pbg_call_sites()     = call_base from errmod_cal on (popbam.cpp:288-306) +
 *                            clean_heterozygotes + segbase + qfilter + cal_site_type + the
 *                            make_<cmd> site store, producing one packed row per position;
 *   - pbg_window_stats()   = calc_diff_matrix + calc_nucdiv / calc_sfs / calc_zns /
 *                            calc_omegamax / calc_wall / calc_diverge / calc_nhaps /
 *                            calc_ehhs / calc_minDxy over any list of windows;
 * pbg_run() chains them for one `popbam <cmd>` invocation and prints the reference's TSV
 * (print_<stat>, byte-identical); the CLI and the tests use it.
 *
 * Conventions: every entry point returns 0 on success or a negative PBG_E* code and never
 * exits; pbg_last_error() has the message.  One context per device; calls on one context are
 * not thread-safe.  Pointers documented "device" must be device (HBM) memory; the caller owns
 * all buffers it passes; the context owns its tables and scratch.  `stream` is a hipStream_t
 * (NULL = default stream); asynchronous entry points only enqueue work on it, and errors the
 * kernels detect (an inconsistent batch) are reported by the next pbg_check() on that stream.
 */
#ifndef POPBAM_GPU_H
#define POPBAM_GPU_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PBG_MAX_SAMPLES 126    /* the reference stops at 64 (u64 masks, popbam.1:507-510,
                                  popbam.cpp:168); 65..126 use the two-word masks below and
                                  16-byte rows (126 sample bits + counted + segregating)  */
#define PBG_MAX_POPS    64     /* pop_mask[] is indexed by population (popbam.1:507-510) */
#define PBG_SITE_BLOCK  64     /* positions per pbg_pileup.block_off entry                 */

#define PBG_OK           0
#define PBG_E_ARG       -1
#define PBG_E_HIP       -2
#define PBG_E_NOMEM     -3
#define PBG_E_RANGE     -4
#define PBG_E_NODEV     -5
#define PBG_E_BATCH     -6     /* a kernel found block_off inconsistent with k[] (pbg_check) */

/* BAM_* option bits, same values as popbam.h:59-94 */
#define PBG_F_ILLUMINA     0x02
#define PBG_F_SUBSTITUTE   0x10
#define PBG_F_HETEROZYGOTE 0x20
#define PBG_F_OUTGROUP     0x40

typedef struct pbg_ctx pbg_ctx;

/* Sample model + calling filters (popbamData members, popbam.h:236-264; defaults
 * popbam.cpp:79-93). */
typedef struct {
    int32_t  n_samples;                 /* sm->n, 1..PBG_MAX_SAMPLES                     */
    int32_t  n_pops;                    /* sm->npops, 1..PBG_MAX_POPS                    */
    uint64_t pop_mask[PBG_MAX_POPS];    /* assign_pops (popbam.cpp:145-171)              */
    int32_t  pop_n[PBG_MAX_POPS];       /* pop_nsmpl                                      */
    int32_t  min_depth, max_depth;      /* -m -x                                          */
    int32_t  min_rmsQ, min_snpQ;        /* -q -s                                          */
    int32_t  min_mapQ, min_baseQ;       /* -a -b (unsigned char in the reference); applied
                                           by the host when it builds the keys            */
    uint32_t flag;                      /* PBG_F_* bits                                   */
    uint64_t pop_mask_hi[PBG_MAX_POPS]; /* samples 64..125 of each pop_mask (0 for n <= 64) */
} pbg_params;

/* Dense pileup batch for contiguous positions [pos0, pos0 + n_sites) of one contig, in the
 * layout SURVEY 8(d) prices (sum over (position, sample) of 2k + 5 bytes, + 1 per position).
 * All pointers are DEVICE pointers for pbg_call_sites, HOST pointers for pbg_run.
 *   ref[i]        reference base byte (faidx_fetch_seq); bit 7 set = the pileup made no
 *                 callback at this position (no mask-passing read covers it)
 *   k[i*n+s]      keys kept for sample s at position i: call_base's `k` after the max_depth
 *                 cap and the per-read filters (popbam.cpp:266-287); u8 when the context's
 *                 max_depth <= 255, else u16 (pbg_k_bytes)
 *   rmsq[i*n+s]   sum of mapQ^2 over those reads (popbam.cpp:287 `rmsq`)
 *   block_off[b]  index in keys[] of the first key of position b*PBG_SITE_BLOCK;
 *                 ceil(n_sites/PBG_SITE_BLOCK)+1 entries, last = total keys (pbg_run derives
 *                 it from k[] when NULL)
 *   keys[]        one u16 per kept read, (position, sample, pileup order) major:
 *                 qq<<5 | strand<<4 | base (popbam.cpp:284), qq = clamp(min(baseQ, mapQ), 4, 63)
 * Device batches: keys[], k[] and rmsq[] must be 16-byte aligned (any hipMalloc / torch
 * allocation is; the kernels read them with 16-byte loads).
 * block_off[0] need not be 0: the kernels read only the 16-byte chunks of keys[] that hold
 * keys [block_off[0], block_off[last]), so a caller may pass keys shifted back by a
 * multiple of 8 keys to address a buffer that holds only that range.                     */
typedef struct {
    uint32_t        n_sites;
    int32_t         pos0;
    const uint8_t  *ref;
    const void     *k;
    const uint32_t *rmsq;
    const uint64_t *block_off;
    const uint16_t *keys;
} pbg_pileup;

/* Row format written by pbg_call_sites: one little-endian word of W = 8*pbg_row_bytes()
 * bits per position (2 B for n<=14, 4 B for n<=30, 8 B for n<=62, 16 B for n<=126):
 *   bits 0..n-1  cal_site_type: sample derived & passing ((cb&3)==3)
 *   bit  W-2     counted: all n samples pass qfilter (popcount(sample_cov)==n)
 *   bit  W-1     segregating: counted and segbase() > 0
 * A position that is not counted has row 0.                                            */

typedef struct { int32_t beg, end; } pbg_window;   /* row index range [beg, end)           */

/* statistics selectable in pbg_window_stats */
#define PBG_S_NUCDIV   0x001   /* pi / dxy              (pop_nucdiv.cpp:206-256)      */
#define PBG_S_SFS      0x002   /* Tajima D, Fay-Wu H    (pop_sfs.cpp:227-291)         */
#define PBG_S_ZNS      0x004   /* ld -o 0               (pop_ld.cpp:201-252)          */
#define PBG_S_OMEGA    0x008   /* ld -o 1               (pop_ld.cpp:254-373)          */
#define PBG_S_WALL     0x010   /* ld -o 2               (pop_ld.cpp:375-458)          */
#define PBG_S_DIV_IND  0x020   /* diverge -o 0          (pop_diverge.cpp:228-231)     */
#define PBG_S_DIV_POP  0x040   /* diverge -o 1          (pop_diverge.cpp:232-253)     */
#define PBG_S_HAP_K    0x080   /* haplo -o 0            (pop_haplo.cpp:208-254)       */
#define PBG_S_HAP_EHHS 0x100   /* haplo -o 1            (pop_haplo.cpp:256-323)       */
#define PBG_S_HAP_DXY  0x200   /* haplo -o 2            (pop_haplo.cpp:325-363)       */
#define PBG_S_TREE     0x400   /* tree diff_matrix      (pop_tree.cpp:472-494)        */

typedef struct {
    uint32_t stats;        /* PBG_S_* mask; at most one of ZNS / OMEGA / WALL (they share
                              ld_snps / ld_val)                                            */
    int32_t  min_freq;     /* ld: 1, or 2 with -e                                         */
    int32_t  outidx;       /* sfs/diverge outgroup sample (-p) when PBG_F_OUTGROUP is set  */
    int32_t  jc;           /* diverge -d jc                                                */
} pbg_stat_opts;

/* Per-window results (DEVICE arrays, caller-allocated, NULL = not wanted).  Values are the
 * exact numbers the reference prints (already divided by num_sites where it divides). */
typedef struct {
    int32_t  *num_sites;   /* [n_win]                                                    */
    int32_t  *segsites;    /* [n_win]                                                    */
    double   *pi;          /* [n_win*n_pops]            nucdiv pi (piw/num_sites)         */
    double   *dxy;         /* [n_win*n_pops*(n_pops-1)] nucdiv dxy, reference indexing    */
    double   *td, *fwh;    /* [n_win*n_pops]            sfs                               */
    int32_t  *ld_snps;     /* [n_win*n_pops]            ld S[] column                     */
    double   *ld_val;      /* [n_win*n_pops]            ZnS / omega_max / Wall B          */
    double   *ld_q;        /* [n_win*n_pops]            Wall Q                            */
    double   *div_ind;     /* [n_win*n_samples]         diverge -o 0 distance             */
    int32_t  *div_fixed;   /* [n_win*n_pops]            diverge -o 1 Fixed (u16 wrap)     */
    int32_t  *div_seg;     /* [n_win*n_pops]            diverge -o 1 Seg                  */
    double   *div_pop;     /* [n_win*n_pops]            diverge -o 1 distance             */
    int32_t  *nhaps;       /* [n_win*n_pops]            haplo K                           */
    double   *hap_val;     /* [n_win*n_pops]            haplo Kdiv (1-hdiv) / EHHS / pi   */
    double   *hap_dxy;     /* [n_win*n_pops*(n_pops-1)] haplo -o 2 dxy                    */
    int32_t  *hap_min;     /* [n_win*n_pops*(n_pops-1)] haplo -o 2 min (u16)              */
    int32_t  *tree_diff;   /* [n_win*(n+1)*(n+1)]       tree diff_matrix (u16 values): taxon 0
                              = the reference (differences = derived count), taxon i+1 =
                              sample i; the neighbour-joining tree is built on the host      */
    /* Not printed by the reference (SURVEY 8(c) "parity unpinned"; north_star asks for them),
     * computed under PBG_S_SFS from calc_sfs's own integers (pop_sfs.cpp:227-240):           */
    int32_t  *sfs_bins;    /* [n_win*n_pops*pbg_sfs_stride()] sfs[j] = segregating sites whose
                              (outgroup-flipped) derived count in the population is j        */
    int32_t  *seg_pop;     /* [n_win*n_pops] S of calc_sfs: sites with 0 < freq < n_pop   */
    double   *theta_w;     /* [n_win*n_pops] Watterson's theta S / a1[n_pop] (a1 of
                              calc_a1, pop_sfs.cpp:511-525), per window (not per site)      */
} pbg_window_out;

/* ---- context ---------------------------------------------------------------------- */
int         pbg_create(pbg_ctx **ctx, int device, const pbg_params *params);
void        pbg_destroy(pbg_ctx *ctx);
const char *pbg_last_error(const pbg_ctx *ctx);   /* ctx may be NULL (last create error)  */
int         pbg_row_bytes(const pbg_ctx *ctx);
int         pbg_k_bytes(const pbg_ctx *ctx);      /* 1 (max_depth <= 255) or 2           */
int         pbg_sfs_stride(const pbg_ctx *ctx);   /* largest population size + 1          */
int         pbg_device_count(void);

/* ---- hot path --------------------------------------------------------------------- */
/* rows: device, n_sites * pbg_row_bytes(); cb: device u64[n_sites*n_samples] or NULL
 * (final consensus words, layout pop_utils.cpp:6-24, for the snp subcommand).           */
int pbg_call_sites(pbg_ctx *ctx, const pbg_pileup *pileup, void *rows, uint64_t *cb, void *stream);

/* The staging capacity of pbg_call_sites (from block_off's last entry) and the workspace
 * plan of pbg_window_stats (from the window list) are computed on the first call and cached
 * per (device pointer, size): steady-state calls on a resident batch enqueue kernels only.
 * A caller that rewrites a window list in place with a different layout must pass a new
 * pointer (or n_win / n_rows) to force a new plan. */
int pbg_window_stats(pbg_ctx *ctx, const void *rows, uint32_t n_rows, const pbg_window *wins,
                     uint32_t n_win, const pbg_stat_opts *opts, const pbg_window_out *out,
                     void *stream);

/* Waits for `stream` and reports what the kernels flagged since the last check: PBG_OK;
 * PBG_E_BATCH when a pileup batch's block_off disagreed with its k[] (the affected blocks
 * were written as uncounted rows and never read past their key range); PBG_E_RANGE when the
 * statistics workspace (windows with more than 256 segregating sites, LD lists; up to 4 GiB)
 * ran out -- the windows that could not get a slice have unset outputs. */
int pbg_check(pbg_ctx *ctx, void *stream);

/* "product" for the shipped build; "bounds" for the PBG_BOUNDS debug build (key loads checked);
 * "experiment" for a timing variant built with experiment switches (tools/variant.sh) -- some of
 * which give wrong results, so nothing may ship or benchmark one as the product. */
const char *pbg_build_info(void);

/* ---- one subcommand end to end ------------------------------------------------------ */
enum { PBG_CMD_SNP = 0, PBG_CMD_HAPLO = 1, PBG_CMD_DIVERGE = 2, PBG_CMD_TREE = 3,
       PBG_CMD_NUCDIV = 4, PBG_CMD_LD = 5, PBG_CMD_SFS = 6 };   /* popbam_func_t (popbam.h:208) */

typedef struct {
    int32_t  cmd;          /* PBG_CMD_*                                                   */
    int32_t  output;       /* -o                                                          */
    int32_t  min_sites;    /* -k                                                          */
    int32_t  min_snps;     /* ld -n                                                       */
    int32_t  min_freq;     /* ld 1 / 2 (-e)                                               */
    int32_t  outidx;       /* -p sample index                                             */
    int32_t  jc;           /* diverge / tree -d jc                                        */
    int32_t  windowed;     /* -w given                                                    */
    int64_t  win_size;     /* bases                                                       */
    int32_t  beg, end;     /* parsed region [beg, end) in contig coordinates              */
    const char *chr_name;
    const char *const *sample_names;
    const char *const *pop_names;
    const char *refid;     /* tree: taxon name of the reference (get_refid, pop_utils.cpp:463-498:
                              the header's first AS: tag value)                              */
    int32_t  ms_windows;   /* snp -o 2 header (print_ms, pop_snp.cpp:114-115, printed before the
                              first window): 0 = this call's window count; > 0 = print it with
                              this total (a block of a longer run that starts the run);
                              < 0 = no header (a later block of a longer run)                */
} pbg_cmd;

/* Runs `popbam <cmd>` over a HOST pileup batch that covers contig positions
 * [pileup->pos0, pileup->pos0 + n_sites) (host pointers; block_off may be NULL and is then
 * derived from k[]): one stream (pbg_stream_*, below) over the 64-position blocks the
 * command's windows touch.  Writes the reference's stdout (TSV) into out (NUL-terminated).
 * Returns the text length, or PBG_E_RANGE with *needed set when cap is too small; the text
 * is then kept by the context and pbg_take_text() copies it without running again.       */
long pbg_run(pbg_ctx *ctx, const pbg_cmd *cmd, const pbg_pileup *host_pileup, char *out,
             size_t cap, size_t *needed);
long pbg_take_text(pbg_ctx *ctx, char *out, size_t cap);

/* print_<stat> for windows whose results were copied to the HOST: `host_out` holds host
 * arrays laid out as pbg_window_out, `wbeg`/`wend` the contig coordinates the reference
 * prints (+1 applied here).  Same return convention as pbg_run.                          */
long pbg_format(const pbg_ctx *ctx, const pbg_cmd *cmd, const pbg_window_out *host_out, uint32_t n_win,
                const int32_t *wbeg, const int32_t *wend, char *out, size_t cap, size_t *needed);

/* ---- streamed runs over HOST batches ------------------------------------------------- */
/* The host side of the pileup callback produces a region's key batch position by position; a
 * stream takes it in pieces, in position order, while the walk goes on (the reference instead
 * re-fetches and re-piles every window, pop_nucdiv.cpp:57-125, and calls each position inside
 * the callback).  Each pushed piece is copied to the device in chunks that alternate between
 * two device slots (the copy of chunk i+1 runs under the call of chunk i) and called into the
 * region's rows; pbg_stream_finish then runs every command's windows (main_<cmd>'s window loop)
 * over those rows and prints their TSV.  Slots, pinned staging, the rows buffer and the window
 * lists (with their statistics plans) belong to the context and serve the next stream: a steady
 * state of streams allocates nothing.  One open stream per context; pbg_run is one stream of
 * one command over one piece.
 *   cmds         the commands to print (all over the same region; the pointers inside them --
 *                names -- must stay valid until pbg_stream_finish); snp -o 0 keeps consensus words
 *   pos0,n_sites the region [pos0, pos0 + n_sites) of contig positions the pieces cover
 *   chunk_sites  positions per device slot (0: about 256 MB of pileup per slot)
 * A piece (host pointers, block_off may be NULL: derived from k[]) starts where the previous
 * one ended and holds a multiple of 64 positions unless it is the last.  Pageable buffers are
 * copied before pbg_stream_push returns; pinned ones (hipHostMalloc / hipHostRegister) are read
 * by DMA asynchronously and must stay unchanged until pbg_stream_finish.                     */
typedef struct pbg_stream pbg_stream;
typedef struct {
    uint64_t h2d_bytes;      /* bytes copied host -> device                                   */
    uint32_t pieces, chunks; /* pushes; device chunks                                          */
    uint32_t pinned_chunks;  /* chunks copied straight from pinned caller buffers              */
    uint32_t _pad;
    double   ms_stage;       /* host: pageable pieces -> pinned staging (threaded memcpy)      */
    double   ms_wait;        /* host: waiting for a slot's previous copy                       */
    double   ms_h2d;         /* device: the chunks' H2D copies (events on the copy stream)     */
    double   ms_call;        /* device: pbg_call_sites per chunk (events on the compute stream) */
    double   ms_finish;      /* host: pbg_stream_finish (wait, statistics, D2H, printing)      */
} pbg_stream_prof;
int  pbg_stream_open(pbg_ctx *ctx, const pbg_cmd *cmds, uint32_t n_cmd, int32_t pos0, uint32_t n_sites,
                     uint32_t chunk_sites, pbg_stream **st);
int  pbg_stream_push(pbg_stream *st, const pbg_pileup *host_piece);
/* The same for a COMPACT piece (rows-only streams: not snp -o 0; max_depth <= 33025): a task
 * (position, sample) whose rmsq[] has bit 31 set is reference-only -- the position is called back
 * (ref bit 7 clear), its reference byte is an upper-case A/C/G/T, it has 1..32 keys and every key
 * shows that base -- and its keys are left out of keys[]: block_off counts the keys present, k[]
 * keeps the task's key count and rmsq[] bits 0..30 its sum of mapQ^2 (qfilter).  The scan settles
 * such a task from k and rmsq alone (it does the same for the full piece's reference-only tasks),
 * so the rows equal the full piece's; the other tasks are exactly as in pbg_stream_push.  About
 * 92 % of the keys of a depth-10 panel belong to reference-only tasks, so the piece crosses PCIe
 * in about a quarter of the bytes.  A flag on a task that cannot be reference-only is reported by
 * pbg_stream_finish (PBG_E_BATCH).  Replaces nothing in the reference: call_base's per-read loop
 * (popbam.cpp:266-287) already walks every key of the task, where the test costs a compare. */
int  pbg_stream_push_compact(pbg_stream *st, const pbg_pileup *host_piece);
int  pbg_stream_finish(pbg_stream *st);   /* waits, checks (PBG_E_BATCH ...), prints every command */
/* command i's text (NUL-terminated); returns its length or PBG_E_RANGE with *needed set       */
long pbg_stream_text(pbg_stream *st, uint32_t i, char *out, size_t cap, size_t *needed);
/* copies the region's packed rows (n_sites * pbg_row_bytes() bytes) into dst, host or device
 * memory (the statistics' input: lets a caller check a streamed run against a resident one)   */
int  pbg_stream_rows(const pbg_stream *st, void *dst, size_t cap);
int  pbg_stream_profile(const pbg_stream *st, pbg_stream_prof *prof);
/* the message of the stream's error (its context's last error; "" when it has none): for a
 * caller that holds the stream but not the context, e.g. a pileup callback                 */
const char *pbg_stream_error(const pbg_stream *st);
void pbg_stream_close(pbg_stream *st);

/* ---- profiling ---------------------------------------------------------------------- */
/* With timing on, every pbg_call_sites records a pair of HIP events on its stream around its
 * dominant kernel (the scan kernel of the rows-only pipeline, the block kernel when
 * consensus words are requested) and one pair around the whole call; pbg_kernel_time waits
 * for the recorded events and returns the summed elapsed milliseconds of each and the number
 * of calls timed.  Turning timing on (again) restarts the count.  No reference counterpart
 * (the reference has no timers).                                                  */
int pbg_set_kernel_timing(pbg_ctx *ctx, int on);
int pbg_kernel_time(pbg_ctx *ctx, double *ms_total, uint32_t *launches);
int pbg_call_time(pbg_ctx *ctx, double *ms_total, uint32_t *launches);

/* ---- synthetic workload (benchmark) ------------------------------------------------- */
/* Counter-based pileup generator (splitmix64 keyed on (seed, contig, position);
 * depth ~ Binomial(2 * mean_depth, 1/2), baseQ 20..40, mapQ 60, ~0.8 % error bases, theta
 * ~1.2 %), written straight into device memory in the pbg_pileup layout with the context's
 * filters applied (the keys the host side of the callback would have built).  Positions
 * [pos0, pos0 + n_sites) of `contig`; block_off is relative to this batch.  A task's reads
 * are a window of a per-seed table of 2^20 random read templates (built on the first call
 * with a seed, which then synchronises `stream` once).  ref / k / rmsq / keys must be 16-byte
 * aligned.                                                                                  */
typedef struct {
    uint64_t seed;
    int32_t  contig;
    int32_t  mean_depth;   /* 1..32                                                       */
    int64_t  pos0;
    uint32_t n_sites;
} pbg_synth_spec;

/* Upper bound on the keys of a batch (n_sites * n * 2 * mean_depth): a keys[] buffer this
 * large lets pbg_synth_pileup run without any host synchronisation.                       */
uint64_t pbg_synth_max_keys(const pbg_ctx *ctx, const pbg_synth_spec *spec);
/* Fills ref / k / rmsq / block_off / keys (device).  keys_cap = capacity of keys[] in keys;
 * a batch that needs more fails at the next pbg_check (PBG_E_BATCH) with no write past it.
 * keys = NULL (keys_cap 0) fills everything but the keys (a counting pass).  n_keys (host,
 * may be NULL) receives the key count and makes the call synchronous.                     */
int pbg_synth_pileup(pbg_ctx *ctx, const pbg_synth_spec *spec, uint8_t *ref, void *k, uint32_t *rmsq,
                     uint64_t *block_off, uint16_t *keys, uint64_t keys_cap, uint64_t *n_keys, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* POPBAM_GPU_H */
