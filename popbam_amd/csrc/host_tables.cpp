// host_tables.cpp -- host-built constant tables the kernels read from HBM.
//
// These are the one-off set-up computations of the reference, done once per context on the
// host because they need x87 long double (expl/logl) exactly as the reference computes them:
//   errmod_init(1.0-0.83) -> cal_coef(depcorr, 0.03)     pop_utils.cpp:203-266
//   LogGamma (integer arguments only)                   gamma.cpp:126-166
//   calc_a1 / calc_a2 / calc_e1 / calc_e2               pop_sfs.cpp:511-571
//   r^2 for every (marg1, marg2, c11) of a population    pop_ld.cpp:239-243 (per pop size)
#include <cmath>
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
    // summed from the top in long double
    for (int q = 1; q < 64; ++q) {
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
    }
    for (int n = 0; n < 256; ++n)
        for (int k = 0; k < 256; ++k) lhet[n << 8 | k] = lC[n << 8 | k] - ln2 * n;
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
