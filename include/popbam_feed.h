/* popbam_feed.h -- C-ABI of the host pileup feeder (libpopbam_feed.so).
 *
 * The host side of the drop-in boundary: reads BGZF/BAM + BAI +
 * FASTA and walks the pileup of a region exactly as the reference's callback sees it,
 * producing the dense batch that pbg_run / pbg_call_sites take (include/popbam_gpu.h).
 * It replaces, for the hot path:
 *   - bgzf.c (block reader), bam.c bam_read1 / bam_calend, bam_index.c bam_fetch
 *     (bam_index.c:943-980: reads overlapping [beg, end) in file order);
 *   - bam_pileup.c bam_plp_push / bam_plp_next / resolve_cigar2 (bam_pileup.c:90-407):
 *     a position gets a callback iff at least one buffered read spans it; reads in push
 *     (file) order; BAM_DEF_MASK (bam.h:123) and the 8000-read maxcnt (bam_pileup.c:375);
 *   - the per-sample partition at the top of popbamData::call_base (popbam.cpp:220-249):
 *     skip is_del / is_refskip / BAM_FUNMAP, skip reads without RG, RG -> sample (unknown RG
 *     falls back to the file-name sample, else the reference's fatal error), first
 *     max_depth reads per sample in pileup order;
 *   - faidx.c fai_fetch of one contig (faidx.c:291; .fai used when present).
 *   - call_base's per-read loop (popbam.cpp:252-287): baseQ (Illumina offset) / mapQ / N
 *     filters, the key qq<<5 | strand<<4 | base, k and sum of mapQ^2 -> the pbg_pileup layout
 *     (pbf_pack, pbf_pileup_keys_mt).
 * Host memory only; no GPU.  Functions return 0 / a non-negative value on success and a
 * negative PBF_E* code on error (message in pbf_last_error()); nothing exits.
 */
#ifndef POPBAM_FEED_H
#define POPBAM_FEED_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define PBF_OK       0
#define PBF_E_IO    -1
#define PBF_E_FORMAT -2
#define PBF_E_ARG   -3
#define PBF_E_RG    -4     /* read group not assigned to a sample (reference: fatal_error) */

typedef struct pbf_bam pbf_bam;

/* one pileup batch over contig positions [pos0, pos0 + n_sites), laid out as pbg_pileup
 * (include/popbam_gpu.h): ref bit 7 = no callback at that position                        */
typedef struct {
    uint32_t  n_sites;
    int32_t   pos0;
    uint8_t  *ref;         /* [n_sites]                                                    */
    uint16_t *depth;       /* [n_sites * n_samples]                                        */
    uint64_t *block_off;   /* [n_sites/64 + 2] reads before each 64-position block         */
    uint32_t *reads;       /* [n_reads] baseQ | mapQ<<8 | nt16<<16 | strand<<20            */
    uint64_t  n_reads;
} pbf_batch;

/* the same batch after call_base's per-read loop, laid out as pbg_pileup */
typedef struct {
    uint32_t  n_sites;
    int32_t   pos0;
    uint8_t  *ref;         /* [n_sites]                                                    */
    void     *k;           /* [n_sites * n_samples] u8 or u16 (pbf_filter.k_bytes)          */
    uint32_t *rmsq;        /* [n_sites * n_samples] sum of mapQ^2 over the kept reads       */
    uint64_t *block_off;   /* [n_sites/64 + 2] keys before each 64-position block           */
    uint16_t *keys;        /* [n_keys] qq<<5 | strand<<4 | base (16-byte aligned)           */
    uint64_t  n_keys;
} pbf_keys;

/* call_base's per-read filters (popbamData members, popbam.h:236-264) */
typedef struct {
    int32_t min_baseQ, min_mapQ;   /* -b / -a as the reference holds them (unsigned char)     */
    int32_t illumina;              /* BAM_ILLUMINA (-i): baseQ > 31 ? baseQ - 31 : 0          */
    int32_t k_bytes;               /* width of k[]: 1 (max_depth <= 255) or 2 (pbg_k_bytes)   */
    int32_t compact;               /* pieces in the compact form of pbg_stream_push_compact: a
                                      reference-only task (1..32 keys, all on the upper-case
                                      A/C/G/T reference base of a called position) gets rmsq bit
                                      31 and no keys (needs max_depth <= 33025)                */
} pbf_filter;

const char *pbf_last_error(void);   /* thread-local */

/* Opens a BAM file and, if present, its index (<path>.bai).  */
int  pbf_open(pbf_bam **out, const char *bam_path);
void pbf_close(pbf_bam *b);
const char *pbf_header_text(const pbf_bam *b);
int  pbf_n_refs(const pbf_bam *b);
const char *pbf_ref_name(const pbf_bam *b, int tid);
int64_t pbf_ref_len(const pbf_bam *b, int tid);
int  pbf_has_index(const pbf_bam *b);

/* Pileup of contig `tid` over [beg, end).  `refseq` is the contig sequence (at least `end`
 * bytes).  Read groups: rg_ids[i] -> rg_sample[i]; reads whose RG is not listed go to
 * `fallback_sample` (>= 0; the reference's file-name sample when the header has no @RG) or
 * fail with PBF_E_RG (-1) when they contribute a base.  The batch's arrays are allocated by
 * the library; release them with pbf_batch_free.                                          */
int  pbf_pileup(pbf_bam *b, int tid, int32_t beg, int32_t end, const char *refseq,
                const char *const *rg_ids, const int32_t *rg_sample, int n_rg, int32_t fallback_sample,
                int n_samples, int max_depth, pbf_batch *out);
void pbf_batch_free(pbf_batch *batch);

/* The pileup the reference's window loop sees over [beg, end), split into `chunk`-position
 * pieces (rounded up to a multiple of 64; <= 0 = 1 Mb) walked by `n_threads` threads, each
 * with its own handle on `bam_path` (the host walk multithreaded by region).
 * The reference fetches and walks every window on its own (pop_nucdiv.cpp:57-125): window k
 * of win_size > 0 is [beg + k*win_size, beg + (k+1)*win_size - 1); win_size = 0 means one walk
 * of [beg, end).  A position's pileup depends only on the reads overlapping it unless a
 * read meets a full buffer (maxcnt 8000, bam_pileup.c:375), so a piece where no read can is
 * walked once; a piece where one can is walked window by window as the reference does.
 * On failure the error is the one of the first failing piece in position order.          */
int  pbf_pileup_mt(const char *bam_path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end,
                   int32_t win_size, const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg,
                   int32_t fallback_sample, int n_samples, int max_depth, pbf_batch *out);

/* call_base's per-read loop (popbam.cpp:252-287) over a raw batch: keeps a read iff
 * baseQ (after the Illumina offset) >= min_baseQ, mapQ >= min_mapQ and its base is A/C/G/T,
 * in pileup order.  Arrays allocated by the library; release with pbf_keys_free.          */
int  pbf_pack(const pbf_batch *raw, int n_samples, const pbf_filter *f, pbf_keys *out);
void pbf_keys_free(pbf_keys *keys);
/* A full key batch (pbf_keys / pbg_pileup layout) in the compact form (pbf_filter.compact):
 * allocated by the library, release with pbf_keys_free.  k_bytes: width of in->k.          */
int  pbf_compact(const pbf_keys *in, int n_samples, int k_bytes, pbf_keys *out);

/* pbf_pileup_mt + pbf_pack, through the piece stream below (pbf_kstream_*) merged into one
 * batch: the raw reads of the whole region are never held at once.  Same batch as
 * pbf_pack(pbf_pileup_mt(...)).                                                           */
int  pbf_pileup_keys_mt(const char *bam_path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end,
                        int32_t win_size, const char *refseq, const char *const *rg_ids, const int32_t *rg_sample, int n_rg,
                        int32_t fallback_sample, int n_samples, int max_depth, const pbf_filter *f,
                        pbf_keys *out);

/* The key batch of a region as a stream of pieces in position order (what pbf_pileup_keys_mt
 * merges): `n_threads` workers, each with its own handle on `bam_path`, walk `chunk`-position
 * pieces ahead of the consumer (at most 2 * n_threads pieces wait), so the consumer can hand
 * each piece to the GPU (pbg_stream_push) while the next ones are walked.  A piece is walked
 * once from its own records (the reads spanning each position in file order: bam_plp's buffer)
 * unless a read can meet a full buffer (maxcnt), then window by window as pbf_pileup_mt does.
 * Records are parsed into one arena per piece and each read group is resolved to its sample
 * once per record.  pbf_kstream_next returns 1 with the next piece (release it with
 * pbf_keys_free), 0 after the last, or the first failing piece's error.  `refseq` must stay
 * valid until pbf_kstream_close.                                                           */
typedef struct pbf_kstream pbf_kstream;
typedef struct {
    double   t_wall;             /* seconds since pbf_kstream_open                            */
    double   t_fetch;            /* thread-seconds: index seek + BGZF inflate + record decode */
    double   t_inflate;          /* ... of which inflate                                      */
    double   t_walk;             /* thread-seconds: pileup walk + call_base's per-read loop   */
    double   t_consumer_wait;    /* seconds pbf_kstream_next waited for a piece               */
    uint64_t bytes_compressed, bytes_inflated, records;
    uint32_t threads, pieces, crowded_pieces, _pad;
} pbf_profile;
int  pbf_kstream_open(const char *bam_path, int n_threads, int32_t chunk, int tid, int32_t beg, int32_t end,
                      int32_t win_size, const char *refseq, const char *const *rg_ids, const int32_t *rg_sample,
                      int n_rg, int32_t fallback_sample, int n_samples, int max_depth, const pbf_filter *f,
                      pbf_kstream **out);
int  pbf_kstream_next(pbf_kstream *ks, pbf_keys *piece);
int  pbf_kstream_profile(pbf_kstream *ks, pbf_profile *prof);
void pbf_kstream_close(pbf_kstream *ks);

/* fai_fetch: the whole sequence of contig `name` (case preserved, line breaks removed).
 * *seq is malloc'ed (NUL-terminated); free with pbf_free.                                 */
int  pbf_fasta_fetch(const char *fa_path, const char *name, char **seq, int64_t *len);
void pbf_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
