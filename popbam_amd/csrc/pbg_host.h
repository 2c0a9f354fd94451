// pbg_host.h -- host-side internals of libpopbam_gpu.so (not part of the C-ABI).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/popbam_gpu.h"

namespace pbg {

void build_errmod_tables(std::vector<double> &fk, std::vector<double> &beta, std::vector<double> &lhet);
// The errmod tables are constants (errmod_init(1.0-0.83) has no input): `make` writes them once
// next to the library (errmod_tables.bin, gen_tables.cpp) and a context reads them back instead
// of recomputing ~2 M x87 expl/logl (~0.2-0.3 s of every fresh process).  Returns false (and the
// caller computes them) when the file is absent, of another layout or fails its checksum, or
// when POPBAM_TABLES=compute.
bool write_errmod_tables(const char *path);
bool load_errmod_tables(const char *path, std::vector<double> &fk, std::vector<double> &beta, std::vector<double> &lhet);
void build_sfs_constants(int n, std::vector<double> &a1, std::vector<double> &a2, std::vector<double> &e1,
                         std::vector<double> &e2);
void build_r2_table(int n_pop, std::vector<double> &t);

// Host copies of one window's results, as print_<stat> needs them.
struct WindowHost {
    int32_t beg = 0, end = 0;       // contig coordinates [beg, end)
    int32_t num_sites = 0, segsites = 0;
    std::vector<double> pi, dxy, td, fwh, ld_val, ld_q, div_ind, div_pop, hap_val, hap_dxy;
    std::vector<int32_t> ld_snps, div_fixed, div_seg, nhaps, hap_min, tree_diff;
    // sfs --theta (pbg_cmd.output bit 0): calc_sfs's S, Watterson's theta and the spectrum
    // sfs[0..n_pop] per population (pop_sfs.cpp:246-263)
    std::vector<int32_t> seg_pop;
    std::vector<double> theta_w;
    std::vector<std::vector<int32_t>> sfs_bins;
};

// print_nucdiv / print_sfs / print_ld / print_diverge / print_haplo (TSV, byte-identical)
void format_window(std::string &out, const pbg_cmd &cmd, int n_samples, int n_pops, uint32_t flag,
                   const WindowHost &w);

// print_popbam_snp (pop_snp.cpp:224-241) for one position's consensus words
void format_snp_site(std::string &out, const pbg_cmd &cmd, int n_samples, int32_t pos, unsigned char refc,
                     const uint64_t *cb);
// sample masks of up to PBG_MAX_SAMPLES bits (the reference's u64 for n <= 64)
typedef unsigned __int128 mask128;
inline int popcount128(mask128 x) { return __builtin_popcountll((uint64_t)x) + __builtin_popcountll((uint64_t)(x >> 64)); }
void format_sweep_site(std::string &out, const pbg_cmd &cmd, int n_pops, const mask128 *pop_mask, uint32_t flag,
                       int32_t pos, mask128 types);
void format_ms_header(std::string &out, int n_samples, int n_pops, const int32_t *pop_n, long n_windows);
void format_ms_window(std::string &out, int n_samples, uint32_t flag, int outidx, int32_t wbeg, int32_t wend,
                      const std::vector<int32_t> &pos, const std::vector<mask128> &types);

}  // namespace pbg
