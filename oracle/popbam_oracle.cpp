// popbam_oracle.cpp -- CPU restatement of the POPBAM 0.3 hot path (TEST INFRASTRUCTURE).
//
// Header comment of popbam_oracle.h applies: only tests/, smoke() and bench.py's
// cpu_baseline leg use this, as the checker.  Every function cites the reference
// file:line it restates (paths relative to /root/reference).  Quirks (SURVEY.md
// Appendix A) are reproduced on purpose.  Pinned against the golden TSVs in tests/golden.
//
// Build: g++ -std=c++17 -O2 -ffp-contract=off (x86-64 SSE math, like the reference's -O2).

#include "popbam_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------- lookup tables
// bam_nt16 -> nt4 (popbam.cpp:9); IUPAC genotype letters (popbam.cpp:11);
// iupac_rev: A/a->0 C/c->1 G/g->2 T/t->3 else 14 (popbam.cpp:33-51).
const int kNt16Nt4[16] = {4, 0, 1, 4, 2, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4};
const char kIupac[16] = {'A', 'M', 'R', 'W', 'N', 'C', 'S', 'Y', 'N', 'N', 'G', 'K', 'N', 'N', 'N', 'T'};
inline unsigned char iupac_rev(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 14;
    }
}
// "=ACMGRSVTWYHKDBN"[bam_nt16_table[c]] for the characters iupac[] can hold
inline char nt16_char(unsigned char c) {
    static const char rev[] = "=ACMGRSVTWYHKDBN";
    int v = 15;
    switch (c & 0xDF) {  // upper-case
        case 'A': v = 1; break; case 'C': v = 2; break; case 'M': v = 3; break; case 'G': v = 4; break;
        case 'R': v = 5; break; case 'S': v = 6; break; case 'V': v = 7; break; case 'T': v = 8; break;
        case 'W': v = 9; break; case 'Y': v = 10; break; case 'H': v = 11; break; case 'K': v = 12; break;
        case 'D': v = 13; break; case 'B': v = 14; break; case 'N': v = 15; break;
        default: v = 15;
    }
    if (c == '=') v = 0;
    return rev[v];
}

inline unsigned popcnt64(uint64_t x) { return (unsigned)__builtin_popcountll(x); }

// Sample masks: the reference's unsigned long long (popbam.cpp:168) holds n <= 64 samples.
// The same algorithm runs here on 128-bit masks so that n <= 126 has a CPU statement too
// (beyond 64 no reference output exists: parity there is unpinned).
typedef unsigned __int128 mask_t;
inline unsigned popcnt(mask_t x) { return popcnt64((uint64_t)x) + popcnt64((uint64_t)(x >> 64)); }
inline mask_t pmask(const orc_params *p, int i) { return ((mask_t)p->pop_mask_hi[i] << 64) | p->pop_mask[i]; }
inline int type_words(const orc_params *p) { return p->n_samples > 64 ? 2 : 1; }   // u64 per types[] entry
inline mask_t load_type(const uint64_t *t, size_t pos, int tw) {
    return tw == 2 ? ((mask_t)t[2 * pos + 1] << 64) | t[2 * pos] : (mask_t)t[pos];
}

// ---------------------------------------------------------------- LogGamma
// gamma.cpp:126-166 (and Gamma, gamma.cpp:11-124).  cal_coef only calls it at integer
// x in [1, 256]; for x < 12 Gamma() reduces an integer argument to y == 1 (so the rational
// approximation returns exactly 1.0) and multiplies up y, y+1, ..., i.e. computes
// (x-1)! by repeated multiplication; for x >= 12 the Abramowitz-Stegun 6.1.41 series.
double log_gamma_int(double x) {
    if (x < 12.0) {
        double y = x;
        int n = static_cast<int>(std::floor(y)) - 1;
        y -= n;                     // == 1.0 for integer x >= 1
        double result = 1.0;        // num/den + 1.0 with z == 0
        for (int i = 0; i < n; i++) result *= y++;
        return std::log(std::fabs(result));
    }
    static const double c[8] = {1.0 / 12.0, -1.0 / 360.0, 1.0 / 1260.0, -1.0 / 1680.0,
                                1.0 / 1188.0, -691.0 / 360360.0, 1.0 / 156.0, -3617.0 / 122400.0};
    double z = 1.0 / (x * x);
    double sum = c[7];
    for (int i = 6; i >= 0; i--) {
        sum *= z;
        sum += c[i];
    }
    double series = sum / x;
    static const double halfLogTwoPi = 0.91893853320467274178032973640562;
    return (x - 0.5) * std::log(x) - x + halfLogTwoPi + series;
}

// ---------------------------------------------------------------- cal_coef
// pop_utils.cpp:203-255, called through errmod_init(1.0-0.83) (pop_nucdiv.cpp:34):
// the float parameter narrows 0.17 (pop_utils.cpp:257).
struct Tables {
    std::vector<double> fk, beta, lhet;
    Tables() : fk(256), beta(256 * 256 * 64), lhet(256 * 256) {
        const double depcorr = (double)(float)(1.0 - 0.83);
        const double eta = 0.03;
        const double kLn2 = 0.69314718055994530942, kLn10 = 2.30258509299404568402;
        fk[0] = 1.0;
        for (int n = 1; n != 256; ++n) fk[n] = std::pow(1.0 - depcorr, n) * (1.0 - eta) + eta;
        std::vector<double> lC(256 * 256, 0.0);
        for (int n = 1; n != 256; ++n) {
            double lgn = log_gamma_int(n + 1);
            for (int k = 1; k <= n; ++k) lC[n << 8 | k] = lgn - log_gamma_int(k + 1) - log_gamma_int(n - k + 1);
        }
        for (int q = 1; q != 64; ++q) {
            double e = std::pow(10.0, -q / 10.0);
            double le = std::log(e);
            double le1 = std::log(1.0 - e);
            for (int n = 1; n <= 255; ++n) {
                double *b = beta.data() + (q << 16 | n << 8);
                long double sum, sum1;
                sum1 = sum = 0.0;
                for (int k = n; k >= 0; --k, sum1 = sum) {
                    sum = sum1 + expl(lC[n << 8 | k] + k * le + (n - k) * le1);
                    b[k] = -10.0 / kLn10 * logl(sum1 / sum);
                }
            }
        }
        for (int n = 0; n < 256; ++n)
            for (int k = 0; k < 256; ++k) lhet[n << 8 | k] = lC[n << 8 | k] - kLn2 * n;
    }
};
const Tables &tables() {
    static Tables t;
    return t;
}

// ---------------------------------------------------------------- errmod_cal
// pop_utils.cpp:280-365.  keys: qual:6 (<<5) | strand:1 (<<4) | base (low 4 bits).
void errmod_cal(unsigned short n, unsigned short *bases, float *q) {
    const Tables &T = tables();
    double bsum[16] = {0};   // aux.fsum only feeds the dead bar_e; omitted
    unsigned c[16] = {0};
    int w[32] = {0};
    std::memset(q, 0, 16 * sizeof(float));
    if (n == 0) return;
    if (n > 255) {
        // ks_shuffle (ksort.h:254-262): j = (rand()/RAND_MAX)*i is integer division, 0
        // except when rand() == RAND_MAX; every step swaps a[0] with a[i-1].
        for (int i = n; i > 1; --i) std::swap(bases[0], bases[i - 1]);
        n = 255;
    }
    std::sort(bases, bases + n);  // ks_introsort: ascending, result independent of algorithm
    for (int j = n - 1; j >= 0; --j) {
        unsigned short b = bases[j];
        int qq = b >> 5 < 4 ? 4 : b >> 5;
        if (qq > 63) qq = 63;
        int k = b & 0x1f;
        bsum[k & 0xf] += T.fk[w[k]] * T.beta[qq << 16 | n << 8 | c[k & 0xf]];
        ++c[k & 0xf];
        ++w[k];
    }
    const int m = 4;
    for (int j = 0; j != m; ++j) {
        float tmp1;
        int tmp2;
        tmp1 = 0.0f;
        tmp2 = 0;
        for (int k = 0; k != m; ++k) {
            if (k == j) continue;
            tmp1 += bsum[k];
            tmp2 += c[k];
        }
        if (tmp2) q[j * m + j] = tmp1;
        for (int k = j + 1; k < m; ++k) {
            int cjk = c[j] + c[k];
            tmp2 = 0;
            tmp1 = 0.0f;
            for (int i = 0; i < m; ++i) {
                if (i == j || i == k) continue;
                tmp1 += bsum[i];
                tmp2 += c[i];
            }
            if (tmp2)
                q[j * m + k] = q[k * m + j] = -4.343 * T.lhet[cjk << 8 | c[k]] + tmp1;
            else
                q[j * m + k] = q[k * m + j] = -4.343 * T.lhet[cjk << 8 | c[k]];
        }
        for (int k = 0; k != m; ++k)
            if (q[j * m + k] < 0.0) q[j * m + k] = 0.0;
    }
}

// ---------------------------------------------------------------- gl2cns  pop_utils.cpp:66-100
uint64_t gl2cns(const float q[16], unsigned short k) {
    unsigned short min_ij = 0;
    float mn = FLT_MAX, mn_next = FLT_MAX;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j) {
            float l = q[i << 2 | j];
            if (l < mn) {
                min_ij = (unsigned short)(i << 2 | j);
                mn_next = mn;
                mn = l;
            } else if (l < mn_next) {
                mn_next = l;
            }
        }
    uint64_t snpq = (uint64_t)((mn_next - mn) + 0.499) << 32;
    uint64_t nr = (uint64_t)k << 16;
    uint64_t g = (uint64_t)min_ij << 8;
    return snpq + nr + g;
}

// x86-64 gcc double -> unsigned long long: NaN yields 0x8000000000000000 (cvttsd2si
// "indefinite" path), which the later <<48 discards.
inline uint64_t d2u64(double d) {
    if (std::isnan(d)) return 0x8000000000000000ULL;
    return (uint64_t)d;
}

// ---------------------------------------------------------------- call_base  popbam.cpp:186-313
// reads already partitioned per sample with the max_depth cap (popbam.cpp:220-249 is the
// host side of the boundary); this is the per-sample part from popbam.cpp:252 on.
void call_base(const orc_params *p, const uint16_t *depth, const uint32_t *reads, uint64_t *cb) {
    std::vector<unsigned short> bases;
    for (int j = 0; j < p->n_samples; ++j) {
        cb[j] = 0;
        int dj = depth[j];
        if (dj == 0) continue;
        bases.assign(dj, 0);
        int rmsq = 0;
        unsigned short k = 0;
        for (int i = 0; i < dj; ++i) {
            uint32_t r = reads[i];
            int tmp_baseQ = r & 0xff;
            int baseQ = (p->flag & 0x02) ? (tmp_baseQ > 31 ? tmp_baseQ - 31 : 0) : tmp_baseQ;
            int mapQ = (r >> 8) & 0xff;
            if (baseQ < p->min_baseQ || mapQ < p->min_mapQ) continue;
            int b = kNt16Nt4[(r >> 16) & 0xf];
            if (b > 3) continue;
            int qq = baseQ < mapQ ? baseQ : mapQ;
            if (qq < 4) qq = 4;
            if (qq > 63) qq = 63;
            bases[k++] = (unsigned short)(qq << 5 | ((r >> 20) & 1) << 4 | b);
            rmsq += mapQ * mapQ;
        }
        reads += dj;
        float q[16];
        errmod_cal(k, bases.data(), q);
        uint64_t rms = d2u64((double)std::sqrt((float)rmsq / k) + 0.499);
        cb[j] = gl2cns(q, k);
        cb[j] |= rms << 48;
    }
}

// ---------------------------------------------------------------- clean_heterozygotes  pop_utils.cpp:170-201
void clean_heterozygotes(int n, uint64_t *cb, int ref, int min_snpq) {
    for (int i = 0; i < n; ++i) {
        unsigned char g = (cb[i] >> 8) & 0xff;
        unsigned char a1 = (g >> 2) & 0x3, a2 = g & 0x3;
        unsigned short sq = (cb[i] >> 32) & 0xffff;
        unsigned char r = iupac_rev((unsigned char)ref);
        int d = (int)a2 - (int)a1;
        if (a1 != a2 && sq >= min_snpq) {
            if (a1 == r) cb[i] += (uint64_t)(int64_t)(d * (1 << 10));
            if (a2 == r) cb[i] -= (uint64_t)(int64_t)(d * (1 << 8));
        }
        if (a1 != a2 && sq < min_snpq) {
            if (a1 != r) cb[i] += (uint64_t)(int64_t)(d * (1 << 10));
            if (a2 != r) cb[i] -= (uint64_t)(int64_t)(d * (1 << 8));
        }
    }
}

// ---------------------------------------------------------------- segbase  pop_utils.cpp:122-168
int segbase(int n, uint64_t *cb, char ref, int min_snpq) {
    int baseCount[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
        unsigned char g = (cb[i] >> 8) & 0xff;
        unsigned char a1 = (g >> 2) & 0x3, a2 = g & 0x3;
        unsigned short sq = (cb[i] >> 32) & 0xffff;
        if (a1 == a2 && kIupac[g] != ref && sq >= min_snpq) {
            cb[i] |= 0x2ULL;
            ++baseCount[a1];
        } else if (a1 == a2 && kIupac[g] != ref && sq < min_snpq) {
            // revert to the reference; the second subtraction borrows (Appendix A.3)
            int d = (int)g - (int)iupac_rev((unsigned char)ref);
            cb[i] -= (uint64_t)(int64_t)(d * (1 << 8));
            cb[i] -= (uint64_t)(int64_t)(d * (1 << 10));
        }
    }
    int j = 0, k = 0;
    for (int i = 0; i < 4; ++i)
        if (baseCount[i] > 0) { ++j; k = i; }
    return j > 1 ? -1 : baseCount[k];
}

// ---------------------------------------------------------------- qfilter  pop_utils.cpp:102-120
mask_t qfilter(int n, uint64_t *cb, int min_rmsQ, int min_depth, int max_depth) {
    mask_t cov = 0;
    for (int i = 0; i < n; ++i) {
        unsigned short rms = (cb[i] >> 48) & 0xffff;
        unsigned short nr = (cb[i] >> 16) & 0xffff;
        if (rms >= min_rmsQ && nr >= min_depth && nr <= max_depth) {
            cb[i] |= 0x1ULL;
            cov |= (mask_t)1 << i;
        }
    }
    return cov;
}

// ---------------------------------------------------------------- per-window state (hData_t)
struct Window {
    int beg = 0, end = 0, num_sites = 0, segsites = 0;
    std::vector<mask_t> types;                 // popbamData::types, per counted site
    std::vector<std::vector<uint64_t>> seq;    // hap.seq[sample][word]
    std::vector<unsigned> idx, pos;            // hap.idx / hap.pos per seg site
    std::vector<std::vector<uint16_t>> snpq, rms, nreads;
    std::vector<std::vector<unsigned char>> gbyte;
    std::vector<char> refc;
};

struct Out {
    std::string s;
    void str(const char *x) { s += x; }
    void str(const std::string &x) { s += x; }
    void i(long long v) { s += std::to_string(v); }
    void f(double v) {  // std::fixed << std::setprecision(5)
        char b[512];
        std::snprintf(b, sizeof b, "%.5f", v);
        s += b;
    }
    void na() { s += "     NA"; }  // std::setw(7) << "NA"
};

std::string popname(const orc_cmd *c, int i) { return c->pop_names[i]; }

// calc_diff_matrix pop_nucdiv.cpp:242-256 (same in pop_haplo.cpp:444-458): u16 wrap
std::vector<std::vector<uint16_t>> diff_matrix(const orc_params *p, const Window &W) {
    int n = p->n_samples;
    std::vector<std::vector<uint16_t>> d(n, std::vector<uint16_t>(n, 0));
    int words = (W.segsites - 1) / 64;  // SEG_IDX (popbam.h:124), C truncation
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++) {
            for (int k = 0; k <= words; k++) d[j][i] += popcnt64(W.seq[i][k] ^ W.seq[j][k]);
            d[i][j] = d[j][i];
        }
    return d;
}

void head(Out &o, const orc_cmd *c, const Window &W) {
    o.str(c->chr_name); o.str("\t"); o.i(W.beg + 1); o.str("\t"); o.i(W.end + 1); o.str("\t"); o.i(W.num_sites);
}

// ---- nucdiv: calc_nucdiv pop_nucdiv.cpp:206-239, print_nucdiv 258-289
void do_nucdiv(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    int np = p->n_pops, n = p->n_samples;
    auto d = diff_matrix(p, W);
    std::vector<double> piw(np, 0.0), pib(np * (np - 1) > 0 ? np * (np - 1) : 1, 0.0);
    for (int i = 0; i < np; i++)
        for (int j = i; j < np; j++) {
            for (int v = 0; v < n - 1; v++)
                for (int w = v + 1; w < n; w++)
                    if ((pmask(p, i) >> v & 1) && (pmask(p, j) >> w & 1)) {
                        if (i == j) piw[i] += (double)d[v][w];
                        else pib[i * np + (j - (i + 1))] += (double)d[v][w];
                    }
            if (i != j)
                pib[i * np + (j - (i + 1))] *= 1.0 / (double)(p->pop_n[i] * p->pop_n[j]);
            else {
                piw[i] *= 2.0 / (double)(p->pop_n[i] * (p->pop_n[i] - 1));
                if (std::isnan(piw[i])) piw[i] = 0.;
            }
        }
    head(o, c, W);
    for (int i = 0; i < np; i++) {
        o.str("\tpi[" + popname(c, i) + "]:\t");
        if (W.num_sites >= c->min_sites) o.f(piw[i] / W.num_sites); else o.na();
    }
    for (int i = 0; i < np - 1; i++)
        for (int j = i + 1; j < np; j++) {
            o.str("\tdxy[" + popname(c, i) + "-" + popname(c, j) + "]:\t");
            if (W.num_sites >= c->min_sites) o.f(pib[i * np + (j - (i + 1))] / W.num_sites); else o.na();
        }
    o.str("\n");
}

// ---- sfs: calc_a1..e2 pop_sfs.cpp:511-571, calc_sfs 227-291, print_sfs 293-317
struct SfsConst { std::vector<double> a1, a2, e1, e2; };
SfsConst sfs_const(int n) {
    SfsConst k;
    k.a1.assign(n + 1, 0); k.a2.assign(n + 2, 0); k.e1.assign(n + 1, 0); k.e2.assign(n + 1, 0);
    k.a1[0] = k.a1[1] = 1.0;
    for (int i = 2; i <= n; i++) { k.a1[i] = 0; for (int j = 1; j < i; j++) k.a1[i] += 1.0 / (double)(j); }
    k.a2[0] = k.a2[1] = 1.0;
    for (int i = 2; i <= n + 1; i++) { k.a2[i] = 0; for (int j = 1; j < i; j++) k.a2[i] += 1.0 / (double)(j * j); }
    k.e1[0] = k.e1[1] = 1.0;
    for (int i = 2; i <= n; i++) {
        double b1 = (i + 1.0) / (3.0 * (i - 1));
        k.e1[i] = (b1 - (1.0 / k.a1[i])) / k.a1[i];
    }
    k.e2[0] = k.e2[1] = 1.0;
    for (int i = 2; i <= n; i++) {
        double b2 = (2.0 * (i * i + i + 3.0)) / (9.0 * i * (i - 1));
        k.e2[i] = (b2 - ((i + 2.0) / (k.a1[i] * i)) + (k.a2[i] / (k.a1[i] * k.a1[i]))) / ((k.a1[i] * k.a1[i]) + k.a2[i]);
    }
    return k;
}

// the SFS of population i and its segregating-site count S (calc_sfs, pop_sfs.cpp:238-254)
void sfs_bins(const orc_params *p, const orc_cmd *c, const Window &W, int i, std::vector<int> &sfs, int &S) {
    sfs.assign(p->pop_n[i] + 1, 0);
    S = 0;
    for (int j = 0; j < W.segsites; j++) {
        mask_t t = W.types[W.idx[j]];
        mask_t pt = t & pmask(p, i);
        unsigned short freq;
        if ((p->flag & 0x40) && (t >> c->outidx & 1)) freq = (unsigned short)(p->pop_n[i] - popcnt(pt));
        else freq = (unsigned short)popcnt(pt);
        ++sfs[freq];
        if (freq > 0 && freq < p->pop_n[i]) ++S;
    }
}

void do_sfs(Out &o, const orc_params *p, const orc_cmd *c, const Window &W, const SfsConst &K) {
    int np = p->n_pops;
    std::vector<double> td(np, 0.0), fwh(np, 0.0);
    std::vector<int> num_snps(np, 0);
    for (int i = 0; i < np; i++) {
        std::vector<int> sfs;
        sfs_bins(p, c, W, i, sfs, num_snps[i]);
        int n = p->pop_n[i];
        int S = num_snps[i];
        if (S > 0 && n > 1) {
            const double *a1 = K.a1.data(), *a2 = K.a2.data(), *e1 = K.e1.data(), *e2 = K.e2.data();
            for (int j = 1; j < n; j++) {
                td[i] += sfs[j] * (((2.0 * j * (n - j)) / (n * (n - 1))) - (1.0 / a1[n]));
                fwh[i] += sfs[j] * ((1.0 / a1[n]) - ((double)j / (n - 1)));
            }
            td[i] /= std::sqrt(e1[n] * S + e2[n] * S * (S - 1));
            fwh[i] /= std::sqrt(((n - 2) * (S / a1[n]) / (6.0 * (n - 1))) +
                                ((S * (S - 1) / ((a1[n] * a1[n]) + a2[n])) *
                                 (18.0 * (n * n) * (3.0 * n + 2.0) * a2[n + 1] - (88.0 * n * n * n + 9.0 * (n * n) - 13.0 * n + 6.0)) /
                                 (9.0 * n * ((n - 1) * (n - 1)))));
        } else {
            td[i] = std::numeric_limits<double>::quiet_NaN();
            fwh[i] = std::numeric_limits<double>::quiet_NaN();
        }
    }
    head(o, c, W);
    for (int i = 0; i < np; i++) {
        o.str("\tD[" + popname(c, i) + "]:\t");
        if (std::isnan(td[i])) o.na(); else o.f(td[i]);
        o.str("\tH[" + popname(c, i) + "]:\t");
        if (std::isnan(fwh[i])) o.na(); else o.f(fwh[i]);
    }
    o.str("\n");
}

// ---- ld: calc_zns pop_ld.cpp:201-252, calc_omegamax 254-373, calc_wall 375-458, print_ld 650-712
inline double r2_of(unsigned m1, unsigned m2, unsigned c11, int n) {
    double x0 = (double)m1 / n, x1 = (double)m2 / n, x11 = (double)c11 / n;
    return ((x11 - x0 * x1) * (x11 - x0 * x1)) / (x0 * (1. - x0) * x1 * (1. - x1));
}

void do_ld(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    int np = p->n_pops;
    int S = W.segsites;
    std::vector<int> num_snps(np, 0);
    std::vector<double> val(np, 0.0), wallq(np, 0.0);
    const int mf = c->min_freq;
    auto var = [&](unsigned m, int i) { return (int)m >= mf && (int)m <= p->pop_n[i] - mf; };
    if (c->output == 1) {  // omega max
        if (S >= 1)
            for (int j = 0; j < np; j++) {
                std::vector<std::vector<double>> r2(S, std::vector<double>(S, 0.0));
                num_snps[j] = 0;
                int count1 = 0, count2 = 0;
                for (int i = 0; i < S - 1; i++) {
                    mask_t t1 = W.types[W.idx[i]] & pmask(p, j);
                    unsigned m1 = popcnt(t1);
                    if (var(m1, j)) {
                        ++num_snps[j];
                        count2 = count1;
                        for (int k = i + 1; k < S; k++) {
                            mask_t t2 = W.types[W.idx[k]] & pmask(p, j);
                            unsigned m2 = popcnt(t2);
                            if (var(m2, j)) {
                                ++count2;
                                r2[count1][count2] = r2_of(m1, m2, popcnt(t1 & t2), p->pop_n[j]);
                                r2[count2][count1] = r2[count1][count2];
                            }
                        }
                        ++count1;
                    }
                }
                ++num_snps[j];
                double sl = 0, sr = 0, sb = 0;
                val[j] = 0;
                int ns = num_snps[j];
                for (int i = 1; i < ns - 1; i++) {
                    for (int k = 0; k < i; k++)
                        for (int m = k + 1; m <= i; m++) sl += r2[k][m];
                    for (int k = i + 1; k < ns; k++)
                        for (int m = 0; m <= i; m++) sb += r2[k][m];
                    for (int k = i + 1; k < ns - 1; k++)
                        for (int m = k + 1; m < ns; m++) sr += r2[k][m];
                    int left = i + 1, right = ns - left;
                    double omega = (sl + sr) / (((left * (left - 1)) / 2.0) + ((right * (right - 1)) / 2.0));
                    omega *= left * right / sb;
                    val[j] = omega > val[j] ? omega : val[j];
                }
            }
    } else if (c->output == 2) {  // Wall's B and Q
        if (S >= 1) {
            mask_t last_type = 0;  // shared across populations (Appendix A.9)
            std::vector<int> cong(np, 0), part(np, 0);
            std::vector<std::vector<mask_t>> uniq(np);
            for (int i = 0; i < S; i++)
                for (int j = 0; j < np; j++) {
                    mask_t t = W.types[W.idx[i]];
                    mask_t type = t & pmask(p, j);
                    mask_t comp = ~t & pmask(p, j);
                    if (type > 0 && type < pmask(p, j)) {
                        if (num_snps[j] == 0) {
                            uniq[j].push_back(type);
                            last_type = type;
                            num_snps[j]++;
                        } else {
                            if (type == last_type || comp == last_type) {
                                cong[j]++;
                                long x = std::count(uniq[j].begin(), uniq[j].end(), type);
                                long y = std::count(uniq[j].begin(), uniq[j].end(), comp);
                                if (x == 0 && y == 0) {
                                    uniq[j].push_back(type);
                                    part[j]++;
                                }
                            }
                            num_snps[j]++;
                            last_type = type;
                        }
                    }
                }
            for (int i = 0; i < np; i++) {
                val[i] = (double)cong[i] / (double)(num_snps[i] - 1);
                wallq[i] = (double)(cong[i] + part[i]) / num_snps[i];
            }
        }
    } else {  // ZnS
        if (S >= 1)
            for (int i = 0; i < np; i++) {
                num_snps[i] = 0;
                for (int j = 0; j < S - 1; j++) {
                    mask_t t1 = W.types[W.idx[j]] & pmask(p, i);
                    unsigned m1 = popcnt(t1);
                    if (var(m1, i)) {
                        ++num_snps[i];
                        for (int k = j + 1; k < S; k++) {
                            mask_t t2 = W.types[W.idx[k]] & pmask(p, i);
                            unsigned m2 = popcnt(t2);
                            if (var(m2, i)) val[i] += r2_of(m1, m2, popcnt(t1 & t2), p->pop_n[i]);
                        }
                    }
                }
                ++num_snps[i];
                val[i] *= 2.0 / (num_snps[i] * (num_snps[i] - 1));
            }
    }
    head(o, c, W);
    for (int i = 0; i < np; i++) {
        o.str("\tS[" + popname(c, i) + "]:\t"); o.i(num_snps[i]);
        bool ok = num_snps[i] >= c->min_snps;
        if (c->output == 1) { o.str("\tomax[" + popname(c, i) + "]:\t"); if (ok) o.f(val[i]); else o.na(); }
        else if (c->output == 2) {
            o.str("\tB[" + popname(c, i) + "]:\t"); if (ok) o.f(val[i]); else o.na();
            o.str("\tQ[" + popname(c, i) + "]:\t"); if (ok) o.f(wallq[i]); else o.na();
        } else { o.str("\tZns[" + popname(c, i) + "]:\t"); if (ok) o.f(val[i]); else o.na(); }
    }
    o.str("\n");
}

// ---- diverge: calc_diverge pop_diverge.cpp:220-257, print_diverge 496-574
void do_diverge(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    int n = p->n_samples, np = p->n_pops;
    head(o, c, W);
    bool ok = W.num_sites >= c->min_sites;
    if (c->output == 0) {
        int words = (W.segsites - 1) / 64;
        for (int i = 0; i < n; i++) {
            uint16_t d = 0;
            for (int j = 0; j <= words; j++) d += (uint16_t)popcnt64(W.seq[i][j]);
            o.str(std::string("\td[") + c->sample_names[i] + "]:\t");
            if (!ok) { o.na(); continue; }
            double pd = (double)d / W.num_sites;
            o.f(c->jc ? -0.75 * std::log(1.0 - pd * (4.0 / 3.0)) : pd);
        }
    } else {
        for (int i = 0; i < np; i++) {
            int segs = 0;
            uint16_t fixed = 0;
            for (int j = 0; j < W.segsites; j++) {
                mask_t t = W.types[W.idx[j]];
                mask_t pt = t & pmask(p, i);
                unsigned short freq;
                if ((p->flag & 0x40) && (t >> c->outidx & 1)) freq = (unsigned short)(p->pop_n[i] - popcnt(pt));
                else freq = (unsigned short)popcnt(pt);
                if (freq > 0 && freq < p->pop_n[i]) ++segs;
                else if (freq == p->pop_n[i]) ++fixed;
            }
            std::string pn = popname(c, i);
            if (!ok) {
                o.str("\tFixed[" + pn + "]:\t"); o.na(); o.str("\tSeg[" + pn + "]:\t"); o.na();
                o.str("\td[" + pn + "]:\t"); o.na();
                continue;
            }
            o.str("\tFixed[" + pn + "]:\t"); o.i(fixed);
            o.str("\tSeg[" + pn + "]:\t"); o.i(segs);
            o.str("\td[" + pn + "]:\t");
            double pd = (p->flag & 0x10) ? (double)fixed / W.num_sites : (double)(fixed + segs) / W.num_sites;
            o.f(c->jc ? -0.75 * std::log(1.0 - pd * (4.0 / 3.0)) : pd);
        }
    }
    o.str("\n");
}

// ---- haplo: calc_nhaps pop_haplo.cpp:208-254, calc_ehhs 256-323, calc_minDxy 325-363,
//             print_haplo 365-442
void do_haplo(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    int n = p->n_samples, np = p->n_pops;
    auto d = diff_matrix(p, W);
    std::vector<int> nhaps(np, 0);
    std::vector<double> hdiv(np, 0.0), ehhs(np, 0.0), piw(np, 0.0);
    int npairs = np * (np - 1) > 0 ? np * (np - 1) : 1;
    std::vector<double> pib(npairs, 0.0);
    std::vector<uint16_t> minDxy(npairs, 0);
    auto nhaps_fn = [&]() {
        for (int i = 0; i < np; i++) {
            int nelem = p->pop_n[i];
            if (nelem > 1) {
                std::vector<int> b;
                for (int j = 0; j < n; j++)
                    if (pmask(p, i) >> j & 1) b.push_back(j);
                // local indices j,k index the GLOBAL diff matrix (Appendix A.11)
                for (int j = 0; j < nelem - 1; j++)
                    for (int k = j + 1; k < nelem; k++)
                        if (d[j][k] == 0 && b[k] > b[j]) b.at(k) = j;
                int ff = 0;
                for (int j = 0; j < (int)b.size(); j++) {
                    int f = (int)std::count(b.begin(), b.end(), j);
                    if (f > 0) ++nhaps[i];
                    ff += f * f;
                }
                double sh = (double)(ff) / (double)(nelem * nelem);
                hdiv[i] = 1.0 - ((1.0 - sh) * (double)(nelem / (nelem - 1)));
            } else {
                nhaps[i] = 1;
                hdiv[i] = 1.0;
            }
        }
    };
    if (c->output == 0) nhaps_fn();
    else if (c->output == 1) {
        nhaps_fn();
        for (int i = 0; i < np; i++) {
            if (p->pop_n[i] < 4) { ehhs[i] = std::numeric_limits<double>::quiet_NaN(); continue; }
            std::list<mask_t> pop_site;
            for (int j = 0; j < W.segsites; j++) {
                mask_t pt = W.types[W.idx[j]] & pmask(p, i);
                unsigned short popf = (unsigned short)popcnt(pt);
                if (popf > 1 && popf < p->pop_n[i] - 1) pop_site.push_back(pt);
            }
            int part_max_count = 0;
            mask_t comp = 0, max_site = 0;
            std::list<mask_t> uniq(pop_site);
            uniq.sort();
            uniq.unique();
            for (mask_t pt : uniq) {
                // ~CHECK_BIT(...) is always non-zero: comp accumulates pop_mask (A.11)
                for (int j = 0; j < n; j++)
                    if (pmask(p, i) >> j & 1) comp |= (mask_t)1 << j;
                int before = (int)pop_site.size();
                pop_site.remove(pt);
                pop_site.remove(comp);
                int after = (int)pop_site.size();
                int part_count = (before - after) + 1;
                if (part_count > part_max_count) { part_max_count = part_count; max_site = pt; }
            }
            unsigned short popf = (unsigned short)popcnt(max_site);
            int pn = p->pop_n[i];
            double sh = (1.0 - ((double)((popf * popf) + ((pn - popf) * (pn - popf))) / (pn * pn))) * (double)(pn / (pn - 1));
            ehhs[i] = hdiv[i] / (1.0 - sh);
        }
    } else {
        for (int i = 0; i < np; i++)
            for (int j = i; j < np; j++) {
                int pi = i * np + (j - (i + 1));
                if (i != j) minDxy[pi] = (uint16_t)0xFFFFFFFFu;  // UINT_MAX into u16 (A.7)
                for (int v = 0; v < n - 1; v++)
                    for (int w = v + 1; w < n; w++)
                        if ((pmask(p, i) >> v & 1) && (pmask(p, j) >> w & 1)) {
                            if (i == j) piw[i] += (double)d[v][w];
                            else {
                                pib[pi] += (double)d[v][w];
                                minDxy[pi] = minDxy[pi] < d[v][w] ? minDxy[pi] : d[v][w];
                            }
                        }
                if (i != j) pib[pi] *= 1.0 / (double)(p->pop_n[i] * p->pop_n[j]);
                else {
                    piw[i] *= 2.0 / (double)(p->pop_n[i] * (p->pop_n[i] - 1));
                    if (std::isnan(piw[i])) piw[i] = 0.0;
                }
            }
    }
    head(o, c, W);
    bool ok = W.num_sites >= c->min_sites;
    if (c->output == 0) {
        for (int i = 0; i < np; i++) {
            std::string pn = popname(c, i);
            if (ok) { o.str("\tK[" + pn + "]:\t"); o.i(nhaps[i]); o.str("\tKdiv[" + pn + "]:\t"); o.f(1.0 - hdiv[i]); }
            else { o.str("\tK[" + pn + "]:\t"); o.na(); o.str("\tKdiv[" + pn + "]:\t"); o.na(); }
        }
    } else if (c->output == 1) {
        for (int i = 0; i < np; i++) {
            o.str("\tEHHS[" + popname(c, i) + "]:\t");
            if (ok && !std::isnan(ehhs[i])) o.f(ehhs[i]); else o.na();
        }
    } else {
        for (int i = 0; i < np; i++) { o.str("\tpi[" + popname(c, i) + "]:\t"); if (ok) o.f(piw[i]); else o.na(); }
        for (int i = 0; i < np - 1; i++)
            for (int j = i + 1; j < np; j++) {
                std::string pp = popname(c, i) + "-" + popname(c, j);
                int pi = i * np + (j - (i + 1));
                if (ok) { o.str("\tdxy[" + pp + "]:\t"); o.f(pib[pi]); o.str("\tmin[" + pp + "]:\t"); o.i(minDxy[pi]); }
                else { o.str("\tdxy[" + pp + "]:\t"); o.na(); o.str("\tmin[" + pp + "]:\t"); o.na(); }
            }
    }
    o.str("\n");
}

// ---- snp -o 0: print_popbam_snp pop_snp.cpp:224-241.  A genotype byte >= 16 (segbase
// borrow) makes the reference read iupac[] out of bounds (UB); we print '?' there and the
// tests mask that column.
void do_snp(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    for (int i = 0; i < W.segsites; i++) {
        o.str(c->chr_name); o.str("\t"); o.i((long long)W.pos[i] + 1); o.str("\t");
        char rc[2] = {nt16_char((unsigned char)W.refc[i]), 0};
        o.str(rc);
        for (int j = 0; j < p->n_samples; j++) {
            unsigned char g = W.gbyte[j][i];
            char bc[2] = {g < 16 ? nt16_char((unsigned char)kIupac[g]) : '?', 0};
            o.str("\t"); o.str(bc);
            o.str("\t"); o.i(W.snpq[j][i]);
            o.str("\t"); o.i(W.rms[j][i]);
            o.str("\t"); o.i(W.nreads[j][i]);
        }
        o.str("\n");
    }
}

// ---- snp -o 1: print_sweep pop_snp.cpp:243-268.  At a counted site every sample passes
// qfilter, so pop_sample_mask = sample_cov & pop_mask = pop_mask.
void do_sweep(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    for (int i = 0; i < W.segsites; i++) {
        o.str(c->chr_name); o.str("\t"); o.i((long long)W.pos[i] + 1);
        const mask_t t = W.types[W.idx[i]];
        for (int j = 0; j < p->n_pops; j++) {
            const mask_t pt = t & pmask(p, j);
            const unsigned short pop_n = (unsigned short)popcnt(pmask(p, j));
            unsigned short freq;
            if ((p->flag & 0x40) && (t >> c->outidx & 1)) freq = (unsigned short)(pop_n - popcnt(pt));
            else freq = (unsigned short)popcnt(pt);
            o.str("\t"); o.i(freq); o.str("\t"); o.i(pop_n);
        }
        o.str("\n");
    }
}

// ---- snp -o 2: print_ms pop_snp.cpp:270-303 (positions as std::setprecision(8) = %.8g)
void do_ms(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    o.str("//\nsegsites: "); o.i(W.segsites); o.str("\npositions: ");
    for (int i = 0; i < W.segsites; i++) {
        char b[64];
        std::snprintf(b, sizeof b, "%.8g ", (double)(unsigned)(W.pos[i] - (unsigned)W.beg) / (W.end - W.beg));
        o.str(b);
    }
    o.str("\n");
    for (int i = 0; i < p->n_samples; i++) {
        for (int j = 0; j < W.segsites; j++) {
            const bool d = (W.seq[i][j / 64] >> (j % 64)) & 1;
            const bool flip = (p->flag & 0x40) && (W.types[W.idx[j]] >> c->outidx & 1);
            o.str(d != flip ? "1" : "0");
        }
        o.str("\n");
    }
    o.str("\n");
}

// print_ms_header pop_snp.cpp:305-317, printed before the first window
void ms_header(Out &o, const orc_params *p, long nwindows) {
    o.str("ms "); o.i(p->n_samples); o.str(" "); o.i(nwindows);
    if (p->n_pops > 1) {
        o.str(" -t 5.0 -I "); o.i(p->n_pops); o.str(" ");
        for (int i = 0; i < p->n_pops; i++) { o.i(p->pop_n[i]); o.str(" "); }
    } else {
        o.str(" -t 5.0 ");
    }
    o.str("\n1350154902\n\n");
}

void call_range(const orc_params *p, uint32_t n_sites, const uint8_t *ref, const uint16_t *depth,
                const uint32_t *reads, uint64_t *cb, mask_t *types, int16_t *fq, uint8_t *flags) {
    const int n = p->n_samples;
    std::vector<uint64_t> tmp(n);
    size_t off = 0;
    for (uint32_t s = 0; s < n_sites; s++) {
        const uint16_t *dp = depth + (size_t)s * n;
        uint64_t *c = cb ? cb + (size_t)s * n : tmp.data();
        size_t tot = 0;
        for (int j = 0; j < n; j++) tot += dp[j];
        uint8_t fl = 0;
        mask_t ty = 0;
        int f = 0;
        if (!(ref[s] & 0x80)) {  // make_<cmd> only runs for positions the pileup called back
            fl |= 1;
            call_base(p, dp, reads + off, c);
            char rch = (char)ref[s];
            if (!(p->flag & 0x20)) clean_heterozygotes(n, c, (int)rch, p->min_snpQ);
            f = segbase(n, c, rch, p->min_snpQ);
            mask_t cov = qfilter(n, c, p->min_rmsQ, p->min_depth, p->max_depth);
            if ((int)popcnt(cov) == n) {
                fl |= 2;
                for (int i = 0; i < n; i++)
                    if ((c[i] & 3ULL) == 3ULL) ty |= (mask_t)1 << i;
                if (f > 0) fl |= 4;
            }
        } else if (cb) {
            for (int j = 0; j < n; j++) c[j] = 0;
        }
        off += tot;
        if (types) types[s] = ty;
        if (fq) fq[s] = (int16_t)f;
        if (flags) flags[s] = fl;
    }
}

void add_site(Window &W, const orc_params *p, uint32_t pos, mask_t ty, uint8_t fl, const uint64_t *cb, char refc) {
    if (!(fl & 2)) return;
    int n = p->n_samples;
    W.types.push_back(ty);
    if (fl & 4) {
        int s = W.segsites;
        for (int i = 0; i < n; i++) {
            if ((size_t)(s / 64) >= W.seq[i].size()) W.seq[i].push_back(0);
            if (ty >> i & 1) W.seq[i][s / 64] |= 0x1ULL << (s % 64);
            if (cb) {
                W.snpq[i].push_back((cb[i] >> 32) & 0xffff);
                W.rms[i].push_back((cb[i] >> 48) & 0xffff);
                W.nreads[i].push_back((cb[i] >> 16) & 0xffff);
                W.gbyte[i].push_back((cb[i] >> 8) & 0xff);
            }
        }
        W.idx.push_back(W.num_sites);
        W.pos.push_back(pos);
        W.refc.push_back(refc);
        W.segsites++;
    }
    W.num_sites++;
}

// ---- tree: calc_diff_matrix pop_tree.cpp:472-494, calc_dist_matrix 496-515, make_nj 208-252,
//      join_tree 254-429, print_tree 439-470.  Pointer rings as tree_init builds them.
struct TNode {
    TNode *next = nullptr, *back = nullptr;
    int index = 0;
    bool tip = false;
    double v = 0.0;
};

void t_print(Out &o, const TNode *p, const TNode *start, const char *refid, const char *const *smpl) {
    if (p->tip) {
        o.str(p->index == 1 ? refid : smpl[p->index - 2]);
    } else {
        o.str("(");
        t_print(o, p->next->back, start, refid, smpl);
        o.str(",");
        t_print(o, p->next->next->back, start, refid, smpl);
        if (p == start) {
            o.str(",");
            t_print(o, p->back, start, refid, smpl);
        }
        o.str(")");
    }
    if (p == start) o.str(";\n");
    else if (p->v < 0) o.str(":0.00000");
    else { o.str(":"); o.f(p->v); }
}

void do_tree(Out &o, const orc_params *p, const orc_cmd *c, const Window &W) {
    const int n = p->n_samples, ntaxa = n + 1;
    if (W.num_sites < c->min_sites || W.segsites < 1) {
        head(o, c, W);
        o.str("\tNA\n");
        return;
    }
    std::vector<std::vector<uint16_t>> diff(ntaxa, std::vector<uint16_t>(ntaxa, 0));
    int words = (W.segsites - 1) / 64;
    for (int i = 0; i < n; i++) {
        for (int k = 0; k <= words; k++) diff[i + 1][0] += popcnt64(W.seq[i][k]);
        diff[0][i + 1] = diff[i + 1][0];
    }
    for (int i = 0; i < n - 1; i++)
        for (int j = i + 1; j < n; j++) {
            for (int k = 0; k <= words; k++) diff[j + 1][i + 1] += popcnt64(W.seq[i][k] ^ W.seq[j][k]);
            diff[i + 1][j + 1] = diff[j + 1][i + 1];
        }
    std::vector<std::vector<double>> x(ntaxa, std::vector<double>(ntaxa, 0.0));
    for (int i = 0; i < ntaxa - 1; i++)
        for (int j = i + 1; j < ntaxa; j++) {
            x[i][j] = (double)diff[i][j] / W.num_sites;
            x[j][i] = x[i][j];
            if (c->jc) {
                x[i][j] = -0.75 * std::log(1.0 - (4.0 * x[i][j] / 3.0));
                x[j][i] = x[i][j];
            }
        }
    // tree_init + make_nj's trim of the last ring + setup_tree
    const int nnodes = 2 * ntaxa - 1;
    std::vector<std::unique_ptr<TNode>> pool;
    std::vector<TNode *> nodep(nnodes);
    auto mk = [&]() { pool.emplace_back(new TNode()); return pool.back().get(); };
    for (int i = 0; i < ntaxa; i++) nodep[i] = mk();
    for (int i = ntaxa; i < nnodes; i++) {
        TNode *q = nullptr, *pp = nullptr;
        for (int j = 1; j <= 3; j++) { pp = mk(); pp->next = q; q = pp; }
        pp->next->next->next = pp;
        nodep[i] = pp;
    }
    nodep[nnodes - 1]->next = nodep[nnodes - 1];
    for (int i = 1; i <= nnodes; i++) {
        TNode *h = nodep[i - 1];
        h->back = nullptr; h->tip = i <= ntaxa; h->index = i; h->v = 0.0;
        if (i > ntaxa)
            for (TNode *q = h->next; q != h; q = q->next) { q->back = nullptr; q->tip = false; q->index = i; }
    }
    auto hookup = [](TNode *a, TNode *b) { a->back = b; b->back = a; };
    std::vector<TNode *> cluster(nodep.begin(), nodep.begin() + ntaxa);
    std::vector<int> enterorder(ntaxa);
    for (int i = 0; i < ntaxa; i++) enterorder[i] = i + 1;
    // join_tree
    for (int i = 0; i < ntaxa - 1; i++)
        for (int j = i + 1; j < ntaxa; j++) {
            double da = (x[i][j] + x[j][i]) / 2.0;
            x[i][j] = da; x[j][i] = da;
        }
    double fotu2 = ntaxa - 2.0, total = 0, tmin, dio, djo, bi, bj, bk, dmin;
    int nextnode = ntaxa + 1, mini = 0, minj = 0;
    std::vector<double> av(ntaxa, 0.0), R(ntaxa);
    for (int nc = 1; nc <= ntaxa - 3; nc++) {
        for (int j = 2; j <= ntaxa; j++)
            for (int i = 0; i <= j - 2; i++) x[j - 1][i] = x[i][j - 1];
        tmin = DBL_MAX;
        for (int i = 0; i < ntaxa; i++) R[i] = 0.0;
        for (int ja = 2; ja <= ntaxa; ja++) {
            int jj = enterorder[ja - 1];
            if (cluster[jj - 1] != nullptr)
                for (int ia = 0; ia <= ja - 2; ia++) {
                    int ii = enterorder[ia];
                    if (cluster[ii - 1] != nullptr) { R[ii - 1] += x[ii - 1][jj - 1]; R[jj - 1] += x[ii - 1][jj - 1]; }
                }
        }
        for (int ja = 2; ja <= ntaxa; ja++) {
            int jj = enterorder[ja - 1];
            if (cluster[jj - 1] != nullptr)
                for (int ia = 0; ia <= ja - 2; ia++) {
                    int ii = enterorder[ia];
                    if (cluster[ii - 1] != nullptr) total = fotu2 * x[ii - 1][jj - 1] - R[ii - 1] - R[jj - 1];
                    if (total < tmin) { tmin = total; mini = ii; minj = jj; }
                }
        }
        dio = 0.0; djo = 0.0;
        for (int i = 0; i < ntaxa; i++) { dio += x[i][mini - 1]; djo += x[i][minj - 1]; }
        dmin = x[mini - 1][minj - 1];
        dio = (dio - dmin) / fotu2;
        djo = (djo - dmin) / fotu2;
        bi = (dmin + dio - djo) * 0.5;
        bj = dmin - bi;
        bi -= av[mini - 1];
        bj -= av[minj - 1];
        hookup(nodep[nextnode - 1]->next, cluster[mini - 1]);
        hookup(nodep[nextnode - 1]->next->next, cluster[minj - 1]);
        cluster[mini - 1]->v = bi; cluster[minj - 1]->v = bj;
        cluster[mini - 1]->back->v = bi; cluster[minj - 1]->back->v = bj;
        cluster[mini - 1] = nodep[nextnode - 1];
        cluster[minj - 1] = nullptr;
        nextnode++;
        av[mini - 1] = dmin * 0.5;
        fotu2 -= 1.0;
        for (int j = 0; j < ntaxa; j++)
            if (cluster[j] != nullptr) {
                double da = (x[mini - 1][j] + x[minj - 1][j]) * 0.5;
                if (mini - j - 1 < 0) x[mini - 1][j] = da;
                if (mini - j - 1 > 0) x[j][mini - 1] = da;
            }
        for (int j = 0; j < ntaxa; j++) { x[minj - 1][j] = 0.0; x[j][minj - 1] = 0.0; }
    }
    int el[3] = {0, 0, 0}, nude = 1;
    for (int i = 1; i <= ntaxa; i++)
        if (cluster[i - 1] != nullptr) { el[nude - 1] = i; nude++; }
    bi = (x[el[0] - 1][el[1] - 1] + x[el[0] - 1][el[2] - 1] - x[el[1] - 1][el[2] - 1]) * 0.5;
    bj = x[el[0] - 1][el[1] - 1] - bi;
    bk = x[el[0] - 1][el[2] - 1] - bi;
    bi -= av[el[0] - 1]; bj -= av[el[1] - 1]; bk -= av[el[2] - 1];
    hookup(nodep[nextnode - 1], cluster[el[0] - 1]);
    hookup(nodep[nextnode - 1]->next, cluster[el[1] - 1]);
    hookup(nodep[nextnode - 1]->next->next, cluster[el[2] - 1]);
    cluster[el[0] - 1]->v = bi; cluster[el[1] - 1]->v = bj; cluster[el[2] - 1]->v = bk;
    cluster[el[0] - 1]->back->v = bi; cluster[el[1] - 1]->back->v = bj; cluster[el[2] - 1]->back->v = bk;
    // make_nj: print from the node the reference taxon hangs on
    TNode *start = nodep[0]->back;
    head(o, c, W);
    o.str("\t");
    t_print(o, start, start, c->refid ? c->refid : "", c->sample_names);
}

void init_window(Window &W, const orc_params *p, int b, int e) {
    int n = p->n_samples;
    W = Window();
    W.beg = b; W.end = e;
    W.seq.assign(n, std::vector<uint64_t>(1, 0));
    W.snpq.assign(n, {}); W.rms.assign(n, {}); W.nreads.assign(n, {}); W.gbyte.assign(n, {});
}

void emit(Out &o, const orc_params *p, const orc_cmd *c, const Window &W, const SfsConst &K) {
    switch (c->cmd) {
        case ORC_NUCDIV: do_nucdiv(o, p, c, W); break;
        case ORC_SFS: do_sfs(o, p, c, W, K); break;
        case ORC_LD: do_ld(o, p, c, W); break;
        case ORC_DIVERGE: do_diverge(o, p, c, W); break;
        case ORC_HAPLO: do_haplo(o, p, c, W); break;
        case ORC_TREE: do_tree(o, p, c, W); break;
        case ORC_SNP:
            if (c->output == 1) do_sweep(o, p, c, W);
            else if (c->output == 2) do_ms(o, p, c, W);
            else do_snp(o, p, c, W);
            break;
        default: break;
    }
}

long finish(const Out &o, char *out, size_t cap) {
    if (o.s.size() + 1 > cap) return -(long)(o.s.size() + 1);
    std::memcpy(out, o.s.c_str(), o.s.size() + 1);
    return (long)o.s.size();
}

}  // namespace

extern "C" {

const double *orc_fk(void) { return tables().fk.data(); }
const double *orc_beta(void) { return tables().beta.data(); }
const double *orc_lhet(void) { return tables().lhet.data(); }

int orc_call_sites(const orc_params *p, uint32_t n_sites, const uint8_t *ref, const uint16_t *depth,
                   const uint32_t *reads, uint64_t *cb, uint64_t *types, int16_t *fq, uint8_t *flags) {
    if (!p || p->n_samples < 1 || p->n_samples > ORC_MAX_SAMPLES) return -1;
    std::vector<mask_t> ty(types ? n_sites : 0);
    call_range(p, n_sites, ref, depth, reads, cb, types ? ty.data() : nullptr, fq, flags);
    const int tw = type_words(p);
    if (types)
        for (uint32_t s = 0; s < n_sites; s++) {
            types[(size_t)s * tw] = (uint64_t)ty[s];
            if (tw == 2) types[2 * (size_t)s + 1] = (uint64_t)(ty[s] >> 64);
        }
    return 0;
}

// main_<cmd> window loop, e.g. pop_nucdiv.cpp:47-124
long orc_run(const orc_params *p, const orc_cmd *c, uint32_t n_sites, const uint8_t *ref,
             const uint16_t *depth, const uint32_t *reads, char *out, size_t cap) {
    if (!p || !c || p->n_samples < 1 || p->n_samples > ORC_MAX_SAMPLES) return -1;
    const int n = p->n_samples;
    int beg = c->beg, end = c->end;
    if (end > (int)n_sites) end = (int)n_sites;
    // per-site calls over [beg, end) (each window's re-fetch yields the same pileup per site)
    size_t off = 0;
    for (int s = 0; s < beg; s++)
        for (int j = 0; j < n; j++) off += depth[(size_t)s * n + j];
    int len = end > beg ? end - beg : 0;
    std::vector<uint64_t> cb((size_t)len * n);
    std::vector<mask_t> types(len);
    std::vector<int16_t> fq(len);
    std::vector<uint8_t> flags(len);
    if (len) call_range(p, (uint32_t)len, ref + beg, depth + (size_t)beg * n, reads + off, cb.data(), types.data(), fq.data(), flags.data());
    long num_windows;
    long long w = c->win_size;
    if (c->windowed) num_windows = ((c->end - c->beg) - 1) / w;
    else { w = c->end - c->beg; num_windows = 1; }
    SfsConst K = sfs_const(n);
    Out o;
    Window W;
    if (c->cmd == ORC_SNP && c->output == 2 && num_windows > 0) ms_header(o, p, num_windows);   // cw == 0 only
    for (long cw = 0; cw < num_windows; cw++) {
        int wb, we;
        if (c->windowed) {  // "chr:beg+cw*w+1-(cw+1)*w+beg-1" through bam_parse_region
            wb = (int)(c->beg + cw * w);
            we = (int)((cw + 1) * w + (c->beg - 1));
        } else { wb = c->beg; we = c->end; }
        init_window(W, p, wb, we);
        for (int pos = wb; pos < we && pos < end; pos++) {
            if (pos < beg) continue;
            int s = pos - beg;
            add_site(W, p, (uint32_t)pos, types[s], flags[s], cb.data() + (size_t)s * n, (char)ref[pos]);
        }
        emit(o, p, c, W, K);
    }
    return finish(o, out, cap);
}

long orc_windows_from_sites(const orc_params *p, const orc_cmd *c, const uint64_t *types,
                            const uint8_t *flags, uint32_t n_win, const int32_t *wbeg,
                            const int32_t *wend, char *out, size_t cap) {
    if (!p || !c) return -1;
    SfsConst K = sfs_const(p->n_samples);
    Out o;
    Window W;
    const int tw = type_words(p);
    for (uint32_t i = 0; i < n_win; i++) {
        init_window(W, p, wbeg[i], wend[i]);
        for (int pos = wbeg[i]; pos < wend[i]; pos++)
            add_site(W, p, (uint32_t)pos, load_type(types, pos, tw), flags[pos], nullptr, 0);
        emit(o, p, c, W, K);
    }
    return finish(o, out, cap);
}

// SFS bins, S and Watterson's theta S / a1[n] per (window, population) -- calc_sfs's integers,
// never printed by the reference (parity unpinned beyond the D / H they feed).
long orc_sfs_windows(const orc_params *p, const orc_cmd *c, const uint64_t *types, const uint8_t *flags,
                     uint32_t n_win, const int32_t *wbeg, const int32_t *wend, int stride, int32_t *bins,
                     int32_t *seg_pop, double *theta_w) {
    if (!p || !c) return -1;
    SfsConst K = sfs_const(p->n_samples);
    Window W;
    const int np = p->n_pops;
    const int tw = type_words(p);
    for (uint32_t w = 0; w < n_win; w++) {
        init_window(W, p, wbeg[w], wend[w]);
        for (int pos = wbeg[w]; pos < wend[w]; pos++)
            add_site(W, p, (uint32_t)pos, load_type(types, pos, tw), flags[pos], nullptr, 0);
        for (int i = 0; i < np; i++) {
            std::vector<int> sfs;
            int S = 0;
            sfs_bins(p, c, W, i, sfs, S);
            for (int j = 0; j < stride; j++) bins[((size_t)w * np + i) * stride + j] = j < (int)sfs.size() ? sfs[j] : 0;
            seg_pop[(size_t)w * np + i] = S;
            theta_w[(size_t)w * np + i] = (double)S / K.a1[p->pop_n[i]];
        }
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- synthetic pileup
// Test-only restatement of the benchmark generator (popbam_amd/csrc/pbg_common.h), so CPU
// parity checks can regenerate any position of the HBM-resident workload.
namespace {
uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint32_t mx32(uint32_t x) {   // lowbias32
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
// per (position, sample) hash and depth draw (pbg_common.h synth_sample_hash / synth_depth)
uint64_t sample_hash(uint64_t h, int s) {
    const uint32_t m = (uint32_t)(s + 1);
    return (uint64_t)mx32((uint32_t)h ^ (m * 0xD1B54Bu)) | ((uint64_t)mx32((uint32_t)(h >> 32) ^ (m * 0x9E3779u)) << 32);
}
int depth_draw(uint64_t hs, int mean_depth) {
    const int nb = 2 * mean_depth;
    const uint32_t b0 = mx32((uint32_t)hs ^ 0x5851F42Du);
    if (nb <= 32) return __builtin_popcount(b0 & (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1u)));
    const uint32_t b1 = mx32((uint32_t)(hs >> 32) ^ 0x4C957F2Du);
    const uint64_t m = nb >= 64 ? ~0ULL : ((1ULL << nb) - 1);
    return __builtin_popcountll(((uint64_t)b0 | ((uint64_t)b1 << 32)) & m);
}
}  // namespace

extern "C" void orc_synth_site(uint64_t seed, int32_t contig, uint64_t pos, int32_t n, int32_t mean_depth,
                               int32_t max_depth, uint8_t *ref, uint16_t *depth, uint32_t *reads,
                               uint32_t *n_reads_out) {
    uint64_t h = sm64(seed ^ sm64(pos ^ ((uint64_t)(uint32_t)contig << 40)));
    int ref_idx = (int)(h & 3);
    int snp = ((h >> 2) & 0x3FF) < 12;
    int alt = (ref_idx + 1 + (int)((((h >> 12) & 0xFFFFu) * 3u) >> 16)) & 3;
    uint32_t f16 = (uint32_t)((h >> 16) & 0xFFFF);
    const uint32_t tseed = (uint32_t)sm64(seed ^ 0x6A09E667F3BCC909ULL);   // read-template table seed
    *ref = (uint8_t)"ACGT"[ref_idx];
    uint32_t nr = 0;
    for (int s = 0; s < n; ++s) {
        uint64_t hs = sample_hash(h, s);
        int d = depth_draw(hs, mean_depth);
        if (d > max_depth) d = max_depth;   // call_base keeps the first max_depth reads (popbam.cpp:241-246)
        depth[s] = (uint16_t)d;
        int a0 = (snp && (uint32_t)(hs & 0xFFFF) < f16) ? alt : ref_idx;
        int a1 = (snp && (uint32_t)((hs >> 16) & 0xFFFF) < f16) ? alt : ref_idx;
        // read r = template entry base + 8 (s + n (r >> 3)) + (r & 7): base = the page of the
        // position's 16,384-position span + 64 x bits 32..37 of the site hash (pbg_common.h
        // synth_tmpl_page / synth_tmpl_base / synth_tmpl_index / synth_tmpl_entry)
        const uint64_t span = (pos >> 14) | ((uint64_t)(uint32_t)contig << 40);
        const uint32_t page = (uint32_t)(sm64(seed ^ 0x243F6A8885A308D3ULL ^ span) & ((1u << 20) / 4096u - 1u)) * 4096u;
        const uint32_t wbase = page + (uint32_t)((h >> 32) & 63u) * 64u;
        // the task's errors (pbg_common.h synth_errors): at most two reads, P(one) =
        // d/128 (1 - (d-1)/128), P(two) = d (d - 1) / 32768 (1 - (d-2)/128), from one hash of the
        // sample hash's lower half
        const uint32_t du = (uint32_t)d, eh = mx32((uint32_t)hs ^ 0x2545F491u);
        const uint32_t dd1 = du * (du > 0u ? du - 1u : 0u);
        const uint32_t eu = eh & 0x3FFFu, p2 = (dd1 * (130u - du)) >> 8, p1 = (du << 7) - dd1;
        const uint32_t ne = eu < p2 ? 2u : (eu < p2 + p1 ? 1u : 0u);
        const uint32_t j1 = (((eh >> 14) & 63u) * du) >> 6;
        uint32_t j2 = j1 + 1u + (du > 1u ? (((eh >> 20) & 63u) * (du - 1u)) >> 6 : 0u);
        if (j2 >= du) j2 -= du;
        const uint32_t e1 = 1u + ((((eh >> 26) & 7u) * 3u) >> 3), e2 = 1u + ((((eh >> 29) & 7u) * 3u) >> 3);
        for (int r = 0; r < d; ++r) {
            const uint32_t idx = wbase + 8u * ((uint32_t)s + (uint32_t)n * ((uint32_t)r >> 3)) + ((uint32_t)r & 7u);
            uint32_t hr = tseed ^ (0x9E3779B9u * (idx + 1u));   // mix32 (lowbias32)
            hr ^= hr >> 16;
            hr *= 0x7FEB352Du;
            hr ^= hr >> 15;
            hr *= 0x846CA68Bu;
            hr ^= hr >> 16;
            int base = (hr & 1) ? a1 : a0;
            if (ne >= 1u && (uint32_t)r == j1) base = (base + (int)e1) & 3;
            if (ne >= 2u && (uint32_t)r == j2) base = (base + (int)e2) & 3;
            uint32_t bq = 20 + ((((hr >> 16) & 0xFFFFu) * 21u) >> 16);
            uint32_t strand = ((hr >> 8) ^ (hr >> 17)) & 1u;
            if (reads) reads[nr] = bq | (60u << 8) | ((1u << base) << 16) | (strand << 20);
            ++nr;
        }
    }
    *n_reads_out = nr;
}

// positions [pos_lo, pos_lo + L) as one raw batch; reads[] needs L * n * min(2D, max_depth)
extern "C" uint64_t orc_synth_batch(uint64_t seed, int32_t contig, uint64_t pos_lo, uint32_t L, int32_t n,
                                    int32_t mean_depth, int32_t max_depth, uint8_t *ref, uint16_t *depth,
                                    uint32_t *reads) {
    uint64_t off = 0;
    for (uint32_t i = 0; i < L; ++i) {
        uint32_t nr = 0;
        orc_synth_site(seed, contig, pos_lo + i, n, mean_depth, max_depth, ref + i, depth + (size_t)i * n,
                       reads + off, &nr);
        off += nr;
    }
    return off;
}

// The genotypes behind the synthetic pileup: per position the reference base, per (position,
// sample) the two haplotype alleles a0 | a1 << 2 that synth_read draws from (test-only: the CPU
// baseline writes a BAM of 100 bp reads from them for the reference binary).
extern "C" void orc_synth_genotypes(uint64_t seed, int32_t contig, uint64_t pos_lo, uint32_t L, int32_t n,
                                    uint8_t *ref, uint8_t *alleles) {
    for (uint32_t i = 0; i < L; ++i) {
        const uint64_t pos = pos_lo + i;
        uint64_t h = sm64(seed ^ sm64(pos ^ ((uint64_t)(uint32_t)contig << 40)));
        int ref_idx = (int)(h & 3);
        int snp = ((h >> 2) & 0x3FF) < 12;
        int alt = (ref_idx + 1 + (int)((((h >> 12) & 0xFFFFu) * 3u) >> 16)) & 3;
        uint32_t f16 = (uint32_t)((h >> 16) & 0xFFFF);
        ref[i] = (uint8_t)"ACGT"[ref_idx];
        for (int s = 0; s < n; ++s) {
            uint64_t hs = sample_hash(h, s);
            int a0 = (snp && (uint32_t)(hs & 0xFFFF) < f16) ? alt : ref_idx;
            int a1 = (snp && (uint32_t)((hs >> 16) & 0xFFFF) < f16) ? alt : ref_idx;
            alleles[(size_t)i * n + s] = (uint8_t)(a0 | (a1 << 2));
        }
    }
}

