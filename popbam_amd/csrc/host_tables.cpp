// host_tables.cpp -- host-built constant tables the kernels read from HBM.
//
// These are the one-off set-up computations of the reference, done once per context on the
// host because they need x87 long double (expl/logl) exactly as the reference computes them:
//   errmod_init(1.0-0.83) -> cal_coef(depcorr, 0.03)     pop_utils.cpp:203-266
//   LogGamma (integer arguments only)                   gamma.cpp:126-166
//   calc_a1 / calc_a2 / calc_e1 / calc_e2               pop_sfs.cpp:511-571
//   r^2 for every (marg1, marg2, c11) of a population    pop_ld.cpp:239-243 (per pop size)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "pbg_host.h"

namespace pbg {

namespace {

// LogGamma at integer x >= 1.  Below 12, Gamma() (gamma.cpp:38-111) reduces an integer x to
// y = 1 where its rational approximation is exactly 1.0, then multiplies 1*2*...*(x-1);
// from 12 up, the Abramowitz-Stegun 6.1.41 asymptotic series (gamma.cpp:138-165).
double lgamma_at(int xi) {
    const double x = (double)xi;
    if (x < 12.0) {
        double prod = 1.0, y = 1.0;
        for (int i = 0; i < xi - 1; ++i) prod *= y++;
        return std::log(std::fabs(prod));
    }
    const double c[8] = {1.0 / 12.0, -1.0 / 360.0, 1.0 / 1260.0, -1.0 / 1680.0,
                         1.0 / 1188.0, -691.0 / 360360.0, 1.0 / 156.0, -3617.0 / 122400.0};
    const double z = 1.0 / (x * x);
    double s = c[7];
    for (int i = 6; i >= 0; --i) s = s * z + c[i];   // two roundings per step (no FMA)
    const double series = s / x;
    const double half_log_two_pi = 0.91893853320467274178032973640562;
    return (x - 0.5) * std::log(x) - x + half_log_two_pi + series;
}

}  // namespace

void build_errmod_tables(std::vector<double> &fk, std::vector<double> &beta, std::vector<double> &lhet) {
    const double depcorr = (double)(float)(1.0 - 0.83);   // errmod_init takes a float
    const double eta = 0.03;
    const double ln2 = 0.69314718055994530942, ln10 = 2.30258509299404568402;
    fk.assign(256, 0.0);
    beta.assign(64u * 256u * 256u, 0.0);
    lhet.assign(256u * 256u, 0.0);
    fk[0] = 1.0;
    for (int n = 1; n < 256; ++n) fk[n] = std::pow(1.0 - depcorr, n) * (1.0 - eta) + eta;

    // log binomial coefficients lC[n][k], 1 <= k <= n (0 elsewhere, as calloc leaves them)
    std::vector<double> lC(256 * 256, 0.0);
    std::vector<double> lg(257);
    for (int x = 1; x <= 256; ++x) lg[x] = lgamma_at(x);
    for (int n = 1; n < 256; ++n)
        for (int k = 1; k <= n; ++k) lC[n << 8 | k] = lg[n + 1] - lg[k + 1] - lg[n - k + 1];

    // beta[q][n][k] = -10 log10( P(X > k) / P(X >= k) ), X ~ Bin(n, 10^(-q/10)),
    // summed from the top in long double.  ~2 M expl + logl on the x87 unit (~0.2-0.3 s on one
    // core, most of a fresh process's context creation): the q planes are independent and each
    // is computed in the reference's order, so they are split over threads (same bits)
    auto plane = [&](int q) {
        const double e = std::pow(10.0, -q / 10.0);
        const double le = std::log(e), le1 = std::log(1.0 - e);
        for (int n = 1; n < 256; ++n) {
            double *row = beta.data() + (q << 16 | n << 8);
            long double above = 0.0L;   // sum over j > k
            for (int k = n; k >= 0; --k) {
                const long double incl = above + expl(lC[n << 8 | k] + k * le + (n - k) * le1);
                row[k] = -10.0 / ln10 * logl(above / incl);
                above = incl;
            }
        }
    };
    const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int q = 1 + t; q < 64; q += nt) plane(q);
        });
    for (int q = 1; q < 64; q += nt) plane(q);
    for (auto &x : th) x.join();
    for (int n = 0; n < 256; ++n)
        for (int k = 0; k < 256; ++k) lhet[n << 8 | k] = lC[n << 8 | k] - ln2 * n;
}

namespace {

constexpr char kTabMagic[8] = {'P', 'B', 'G', 'T', 'A', 'B', '0', '1'};
struct TabHeader {
    char magic[8];
    uint64_t n_fk, n_beta, n_lhet;
    uint64_t checksum;   // over the three arrays' bytes, in file order
};

uint64_t checksum_of(const std::vector<const std::vector<double> *> &parts) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (const auto *v : parts)
        for (double d : *v) {
            uint64_t w;
            std::memcpy(&w, &d, 8);
            h = (h ^ w) * 0x100000001B3ull;
            h ^= h >> 29;
        }
    return h;
}

}  // namespace

bool write_errmod_tables(const char *path) {
    std::vector<double> fk, beta, lhet;
    build_errmod_tables(fk, beta, lhet);
    TabHeader h;
    std::memcpy(h.magic, kTabMagic, 8);
    h.n_fk = fk.size(), h.n_beta = beta.size(), h.n_lhet = lhet.size();
    h.checksum = checksum_of({&fk, &beta, &lhet});
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1;
    for (const auto *v : {&fk, &beta, &lhet}) ok = ok && std::fwrite(v->data(), 8, v->size(), f) == v->size();
    return std::fclose(f) == 0 && ok;
}

bool load_errmod_tables(const char *path, std::vector<double> &fk, std::vector<double> &beta,
                        std::vector<double> &lhet) {
    const char *mode = std::getenv("POPBAM_TABLES");
    if (mode && !std::strcmp(mode, "compute")) return false;
    FILE *f = path ? std::fopen(path, "rb") : nullptr;
    if (!f) return false;
    TabHeader h;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && !std::memcmp(h.magic, kTabMagic, 8) && h.n_fk == 256 &&
              h.n_beta == 64u * 256u * 256u && h.n_lhet == 256u * 256u;
    if (ok) {
        fk.resize(h.n_fk), beta.resize(h.n_beta), lhet.resize(h.n_lhet);
        for (auto *v : {&fk, &beta, &lhet}) ok = ok && std::fread(v->data(), 8, v->size(), f) == v->size();
        ok = ok && std::fgetc(f) == EOF && checksum_of({&fk, &beta, &lhet}) == h.checksum;
    }
    std::fclose(f);
    return ok;
}

void build_sfs_constants(int n, std::vector<double> &a1, std::vector<double> &a2, std::vector<double> &e1,
                         std::vector<double> &e2) {
    a1.assign(n + 1, 0.0);
    a2.assign(n + 2, 0.0);
    e1.assign(n + 1, 0.0);
    e2.assign(n + 1, 0.0);
    a1[0] = 1.0;
    if (n >= 1) a1[1] = 1.0;
    for (int i = 2; i <= n; ++i)
        for (int j = 1; j < i; ++j) a1[i] += 1.0 / (double)j;
    a2[0] = a2[1] = 1.0;
    for (int i = 2; i <= n + 1; ++i)
        for (int j = 1; j < i; ++j) a2[i] += 1.0 / (double)(j * j);
    e1[0] = 1.0;
    if (n >= 1) e1[1] = 1.0;
    for (int i = 2; i <= n; ++i) {
        const double b1 = (i + 1.0) / (3.0 * (i - 1));
        e1[i] = (b1 - (1.0 / a1[i])) / a1[i];
    }
    e2[0] = 1.0;
    if (n >= 1) e2[1] = 1.0;
    for (int i = 2; i <= n; ++i) {
        const double b2 = (2.0 * (i * i + i + 3.0)) / (9.0 * i * (i - 1));
        e2[i] = (b2 - ((i + 2.0) / (a1[i] * i)) + (a2[i] / (a1[i] * a1[i]))) / ((a1[i] * a1[i]) + a2[i]);
    }
}

void build_r2_table(int np, std::vector<double> &t) {
    const int m = np + 1;
    t.assign((size_t)m * m * m, 0.0);
    for (int m1 = 0; m1 <= np; ++m1)
        for (int m2 = 0; m2 <= np; ++m2)
            for (int c = 0; c <= np; ++c) {
                const double x0 = (double)m1 / np, x1 = (double)m2 / np, x11 = (double)c / np;
                t[((size_t)m1 * m + m2) * m + c] =
                    ((x11 - x0 * x1) * (x11 - x0 * x1)) / (x0 * (1. - x0) * x1 * (1. - x1));
            }
}

}  // namespace pbg
