// format.cpp -- TSV writer, byte-identical to the reference's print_<stat> functions.
//
// The reference streams to std::cout with `std::fixed << std::setprecision(5)` (sticky),
// which libstdc++ renders through printf's "%.5f"; "NA" cells are `"\t" << std::setw(7) <<
// "NA"`, i.e. five spaces then NA.  Integers print in decimal.
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "pbg_host.h"

namespace pbg {

namespace {

struct W {
    std::string &s;
    void t(const char *x) { s += x; }
    void t(const std::string &x) { s += x; }
    void i(long long v) { s += std::to_string(v); }
    void f(double v) {
        char b[400];
        std::snprintf(b, sizeof b, "%.5f", v);
        s += b;
    }
    void na() { s += "     NA"; }
};

std::string pn(const pbg_cmd &c, int i) { return c.pop_names[i]; }

// ---- tree (pop_tree.cpp): distances, neighbour joining and the Newick printer.
// The tree is O(ntaxa^3) scalar work on an (n+1)x(n+1) matrix per window, so it runs on the
// host on the GPU's diff_matrix.  Nodes live in one array; a ring of three nodes is one
// internal node as in tree_init (pop_tree.cpp:517-539), -1 is the null pointer.
struct NjNode {
    int next = -1, back = -1, index = 0;
    bool tip = false;
    double v = 0.0;
};

struct Nj {
    int ntaxa;
    std::vector<NjNode> nd;
    std::vector<int> nodep;   // curtree.nodep

    explicit Nj(int nt) : ntaxa(nt) {
        const int nnodes = 2 * nt - 1;
        nodep.resize(nnodes);
        for (int i = 0; i < nnodes; ++i) {
            const int h = (int)nd.size();
            if (i < nt) {
                nd.emplace_back();
            } else {   // ring head -> a -> b -> head
                nd.resize(nd.size() + 3);
                nd[h].next = h + 1;
                nd[h + 1].next = h + 2;
                nd[h + 2].next = h;
            }
            nodep[i] = h;
        }
        nd[nodep[nnodes - 1]].next = nodep[nnodes - 1];   // make_nj: last ring cut to one node
        for (int i = 1; i <= nnodes; ++i) {                // setup_tree pop_tree.cpp:541-566
            NjNode &q = nd[nodep[i - 1]];
            q.back = -1;
            q.tip = i <= nt;
            q.index = i;
            q.v = 0.0;
            if (i > nt)
                for (int r = q.next; r != nodep[i - 1]; r = nd[r].next) {
                    nd[r].back = -1;
                    nd[r].tip = false;
                    nd[r].index = i;
                }
        }
    }
    void hookup(int p, int q) {
        nd[p].back = q;
        nd[q].back = p;
    }
    void set_len(int c, double v) {
        nd[c].v = v;
        nd[nd[c].back].v = v;
    }

    // join_tree pop_tree.cpp:254-429, statement for statement (including `total` carried over
    // from a skipped pair and across cycles, and the column sums over cleared rows)
    void join(std::vector<double> x) {
        const int nt = ntaxa;
        auto X = [&](int i, int j) -> double & { return x[(size_t)i * nt + j]; };
        std::vector<int> cluster(nt), eo(nt);
        std::vector<double> av(nt, 0.0), R(nt);
        for (int i = 0; i < nt; ++i) {
            cluster[i] = nodep[i];
            eo[i] = i + 1;
        }
        for (int i = 0; i < nt - 1; i++)
            for (int j = i + 1; j < nt; j++) {
                const double da = (X(i, j) + X(j, i)) / 2.0;
                X(i, j) = da;
                X(j, i) = da;
            }
        double fotu2 = nt - 2.0, total = 0, tmin, dio, djo, bi, bj, bk, dmin;
        int nextnode = nt + 1, mini = 0, minj = 0;
        for (int nc = 1; nc <= nt - 3; nc++) {
            for (int j = 2; j <= nt; j++)
                for (int i = 0; i <= j - 2; i++) X(j - 1, i) = X(i, j - 1);
            tmin = DBL_MAX;
            for (int i = 0; i < nt; i++) R[i] = 0.0;
            for (int ja = 2; ja <= nt; ja++) {
                const int jj = eo[ja - 1];
                if (cluster[jj - 1] < 0) continue;
                for (int ia = 0; ia <= ja - 2; ia++) {
                    const int ii = eo[ia];
                    if (cluster[ii - 1] >= 0) {
                        R[ii - 1] += X(ii - 1, jj - 1);
                        R[jj - 1] += X(ii - 1, jj - 1);
                    }
                }
            }
            for (int ja = 2; ja <= nt; ja++) {
                const int jj = eo[ja - 1];
                if (cluster[jj - 1] < 0) continue;
                for (int ia = 0; ia <= ja - 2; ia++) {
                    const int ii = eo[ia];
                    if (cluster[ii - 1] >= 0) total = fotu2 * X(ii - 1, jj - 1) - R[ii - 1] - R[jj - 1];
                    if (total < tmin) {
                        tmin = total;
                        mini = ii;
                        minj = jj;
                    }
                }
            }
            dio = 0.0;
            djo = 0.0;
            for (int i = 0; i < nt; i++) {
                dio += X(i, mini - 1);
                djo += X(i, minj - 1);
            }
            dmin = X(mini - 1, minj - 1);
            dio = (dio - dmin) / fotu2;
            djo = (djo - dmin) / fotu2;
            bi = (dmin + dio - djo) * 0.5;
            bj = dmin - bi;
            bi -= av[mini - 1];
            bj -= av[minj - 1];
            const int h = nodep[nextnode - 1];
            hookup(nd[h].next, cluster[mini - 1]);
            hookup(nd[nd[h].next].next, cluster[minj - 1]);
            set_len(cluster[mini - 1], bi);
            set_len(cluster[minj - 1], bj);
            cluster[mini - 1] = h;
            cluster[minj - 1] = -1;
            nextnode++;
            av[mini - 1] = dmin * 0.5;
            fotu2 -= 1.0;
            for (int j = 0; j < nt; j++)
                if (cluster[j] >= 0) {
                    const double da = (X(mini - 1, j) + X(minj - 1, j)) * 0.5;
                    if (mini - j - 1 < 0) X(mini - 1, j) = da;
                    if (mini - j - 1 > 0) X(j, mini - 1) = da;
                }
            for (int j = 0; j < nt; j++) {
                X(minj - 1, j) = 0.0;
                X(j, minj - 1) = 0.0;
            }
        }
        int el[3] = {0, 0, 0}, nude = 1;
        for (int i = 1; i <= nt && nude <= 3; i++)
            if (cluster[i - 1] >= 0) el[nude++ - 1] = i;
        bi = (X(el[0] - 1, el[1] - 1) + X(el[0] - 1, el[2] - 1) - X(el[1] - 1, el[2] - 1)) * 0.5;
        bj = X(el[0] - 1, el[1] - 1) - bi;
        bk = X(el[0] - 1, el[2] - 1) - bi;
        bi -= av[el[0] - 1];
        bj -= av[el[1] - 1];
        bk -= av[el[2] - 1];
        const int h = nodep[nextnode - 1];
        hookup(h, cluster[el[0] - 1]);
        hookup(nd[h].next, cluster[el[1] - 1]);
        hookup(nd[nd[h].next].next, cluster[el[2] - 1]);
        set_len(cluster[el[0] - 1], bi);
        set_len(cluster[el[1] - 1], bj);
        set_len(cluster[el[2] - 1], bk);
    }

    // print_tree pop_tree.cpp:439-470
    void print(W &o, int p, int start, const char *refid, const char *const *names) const {
        const NjNode &q = nd[p];
        if (q.tip) {
            o.t(q.index == 1 ? refid : names[q.index - 2]);
        } else {
            o.t("(");
            print(o, nd[q.next].back, start, refid, names);
            o.t(",");
            print(o, nd[nd[q.next].next].back, start, refid, names);
            if (p == start) {
                o.t(",");
                print(o, q.back, start, refid, names);
            }
            o.t(")");
        }
        if (p == start) {
            o.t(";");
        } else if (q.v < 0) {
            o.t(":0.00000");
        } else {
            o.t(":");
            o.f(q.v);
        }
    }
};

// make_nj pop_tree.cpp:208-252 after calc_dist_matrix 496-515 (the caller prints the row head)
void format_nj(W &o, const pbg_cmd &c, int n, const WindowHost &w) {
    if (w.num_sites < c.min_sites || w.segsites < 1) {
        o.t("\tNA");
        return;
    }
    const int nt = n + 1;
    std::vector<double> dist((size_t)nt * nt, 0.0);
    for (int i = 0; i < nt - 1; i++)
        for (int j = i + 1; j < nt; j++) {
            double d = (double)w.tree_diff[(size_t)i * nt + j] / w.num_sites;
            if (c.jc) d = -0.75 * std::log(1.0 - (4.0 * d / 3.0));
            dist[(size_t)i * nt + j] = d;
            dist[(size_t)j * nt + i] = d;
        }
    Nj t(nt);
    t.join(dist);
    const int start = t.nd[t.nodep[0]].back;
    o.t("\t");
    t.print(o, start, start, c.refid ? c.refid : "", c.sample_names);
}

}  // namespace

void format_window(std::string &out, const pbg_cmd &c, int n, int np, uint32_t flag, const WindowHost &w) {
    W o{out};
    o.t(c.chr_name);
    o.t("\t");
    o.i(w.beg + 1);
    o.t("\t");
    o.i(w.end + 1);
    o.t("\t");
    o.i(w.num_sites);
    const bool ok = w.num_sites >= c.min_sites;
    switch (c.cmd) {
        case PBG_CMD_NUCDIV:  // print_nucdiv pop_nucdiv.cpp:258-289
            for (int i = 0; i < np; i++) {
                o.t("\tpi[" + pn(c, i) + "]:\t");
                if (ok) o.f(w.pi[i]); else o.na();
            }
            for (int i = 0; i < np - 1; i++)
                for (int j = i + 1; j < np; j++) {
                    o.t("\tdxy[" + pn(c, i) + "-" + pn(c, j) + "]:\t");
                    if (ok) o.f(w.dxy[i * np + (j - (i + 1))]); else o.na();
                }
            break;
        case PBG_CMD_SFS:  // print_sfs pop_sfs.cpp:293-317 (NA only for NaN)
            for (int i = 0; i < np; i++) {
                o.t("\tD[" + pn(c, i) + "]:\t");
                if (std::isnan(w.td[i])) o.na(); else o.f(w.td[i]);
                o.t("\tH[" + pn(c, i) + "]:\t");
                if (std::isnan(w.fwh[i])) o.na(); else o.f(w.fwh[i]);
            }
            // --theta: the integers and theta_W calc_sfs computes but print_sfs never prints,
            // appended after the reference's columns so the default output is unchanged
            if ((c.output & 1) && (int)w.seg_pop.size() == np && (int)w.sfs_bins.size() == np)
                for (int i = 0; i < np; i++) {
                    o.t("\tS[" + pn(c, i) + "]:\t");
                    o.i(w.seg_pop[i]);
                    o.t("\tthetaW[" + pn(c, i) + "]:\t");
                    if (!std::isfinite(w.theta_w[i])) o.na(); else o.f(w.theta_w[i]);
                    o.t("\tsfs[" + pn(c, i) + "]:\t");
                    for (size_t j = 0; j < w.sfs_bins[i].size(); j++) {
                        if (j) o.t(",");
                        o.i(w.sfs_bins[i][j]);
                    }
                }
            break;
        case PBG_CMD_LD:  // print_ld pop_ld.cpp:650-712
            for (int i = 0; i < np; i++) {
                o.t("\tS[" + pn(c, i) + "]:\t");
                o.i(w.ld_snps[i]);
                const bool sok = w.ld_snps[i] >= c.min_snps;
                if (c.output == 1) {
                    o.t("\tomax[" + pn(c, i) + "]:\t");
                    if (sok) o.f(w.ld_val[i]); else o.na();
                } else if (c.output == 2) {
                    o.t("\tB[" + pn(c, i) + "]:\t");
                    if (sok) o.f(w.ld_val[i]); else o.na();
                    o.t("\tQ[" + pn(c, i) + "]:\t");
                    if (sok) o.f(w.ld_q[i]); else o.na();
                } else {
                    o.t("\tZns[" + pn(c, i) + "]:\t");
                    if (sok) o.f(w.ld_val[i]); else o.na();
                }
            }
            break;
        case PBG_CMD_DIVERGE:  // print_diverge pop_diverge.cpp:496-574
            if (c.output == 0) {
                for (int i = 0; i < n; i++) {
                    o.t(std::string("\td[") + c.sample_names[i] + "]:\t");
                    if (ok) o.f(w.div_ind[i]); else o.na();
                }
            } else {
                for (int i = 0; i < np; i++) {
                    const std::string p = pn(c, i);
                    if (ok) {
                        o.t("\tFixed[" + p + "]:\t");
                        o.i(w.div_fixed[i]);
                        o.t("\tSeg[" + p + "]:\t");
                        o.i(w.div_seg[i]);
                        o.t("\td[" + p + "]:\t");
                        o.f(w.div_pop[i]);
                    } else {
                        o.t("\tFixed[" + p + "]:\t");
                        o.na();
                        o.t("\tSeg[" + p + "]:\t");
                        o.na();
                        o.t("\td[" + p + "]:\t");
                        o.na();
                    }
                }
            }
            (void)flag;
            break;
        case PBG_CMD_HAPLO:  // print_haplo pop_haplo.cpp:365-442
            if (c.output == 0) {
                for (int i = 0; i < np; i++) {
                    const std::string p = pn(c, i);
                    o.t("\tK[" + p + "]:\t");
                    if (ok) o.i(w.nhaps[i]); else o.na();
                    o.t("\tKdiv[" + p + "]:\t");
                    if (ok) o.f(w.hap_val[i]); else o.na();
                }
            } else if (c.output == 1) {
                for (int i = 0; i < np; i++) {
                    o.t("\tEHHS[" + pn(c, i) + "]:\t");
                    if (ok && !std::isnan(w.hap_val[i])) o.f(w.hap_val[i]); else o.na();
                }
            } else {
                for (int i = 0; i < np; i++) {
                    o.t("\tpi[" + pn(c, i) + "]:\t");
                    if (ok) o.f(w.hap_val[i]); else o.na();
                }
                for (int i = 0; i < np - 1; i++)
                    for (int j = i + 1; j < np; j++) {
                        const std::string pp = pn(c, i) + "-" + pn(c, j);
                        const int k = i * np + (j - (i + 1));
                        o.t("\tdxy[" + pp + "]:\t");
                        if (ok) o.f(w.hap_dxy[k]); else o.na();
                        o.t("\tmin[" + pp + "]:\t");
                        if (ok) o.i(w.hap_min[k]); else o.na();
                    }
            }
            break;
        case PBG_CMD_TREE:
            format_nj(o, c, n, w);
            break;
        default:
            break;
    }
    out += "\n";
}

namespace {
// "=ACMGRSVTWYHKDBN"[bam_nt16_table[c]] (popbam.cpp:13-31) for letters
char nt16_letter(unsigned char c) {
    static const char rev[] = "=ACMGRSVTWYHKDBN";
    static const char *letters = "ACMGRSVTWYHKDBN";
    unsigned char u = (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c;
    if (u == '=') return '=';
    for (int i = 0; letters[i]; ++i)
        if (letters[i] == (char)u) return rev[i + 1];
    return 'N';
}
const char kIupac[16] = {'A', 'M', 'R', 'W', 'N', 'C', 'S', 'Y', 'N', 'N', 'G', 'K', 'N', 'N', 'N', 'T'};
}  // namespace

void format_snp_site(std::string &out, const pbg_cmd &c, int n, int32_t pos, unsigned char refc, const uint64_t *cb) {
    W o{out};
    o.t(c.chr_name);
    o.t("\t");
    o.i((long long)pos + 1);
    o.t("\t");
    out += nt16_letter(refc);
    for (int j = 0; j < n; j++) {
        const unsigned g = (unsigned)(cb[j] >> 8) & 0xff;
        // genotype bytes >= 16 only arise from segbase's borrow; the reference then reads
        // iupac[] out of bounds (undefined); we print 'N'
        out += "\t";
        out += g < 16 ? nt16_letter((unsigned char)kIupac[g]) : 'N';
        o.t("\t");
        o.i((long long)((cb[j] >> 32) & 0xffff));
        o.t("\t");
        o.i((long long)((cb[j] >> 48) & 0xffff));
        o.t("\t");
        o.i((long long)((cb[j] >> 16) & 0xffff));
    }
    out += "\n";
}

// snp -o 1: print_sweep (pop_snp.cpp:243-268).  At a counted site every sample passes
// qfilter, so the reference's pop_sample_mask (sample_cov & pop_mask) is pop_mask.
void format_sweep_site(std::string &out, const pbg_cmd &c, int np, const mask128 *pop_mask, uint32_t flag,
                       int32_t pos, mask128 types) {
    W o{out};
    o.t(c.chr_name);
    o.t("\t");
    o.i((long long)pos + 1);
    for (int j = 0; j < np; j++) {
        const mask128 pt = types & pop_mask[j];
        const unsigned pop_n = (unsigned)popcount128(pop_mask[j]);
        const bool flip = (flag & PBG_F_OUTGROUP) && ((types >> c.outidx) & 1);
        const unsigned freq = (unsigned short)(flip ? pop_n - (unsigned)popcount128(pt) : (unsigned)popcount128(pt));
        o.t("\t");
        o.i(freq);
        o.t("\t");
        o.i(pop_n);
    }
    out += "\n";
}

// snp -o 2: print_ms_header (pop_snp.cpp:305-317), once before the first window
void format_ms_header(std::string &out, int n, int np, const int32_t *pop_n, long nwindows) {
    W o{out};
    o.t("ms ");
    o.i(n);
    o.t(" ");
    o.i(nwindows);
    if (np > 1) {
        o.t(" -t 5.0 -I ");
        o.i(np);
        o.t(" ");
        for (int i = 0; i < np; i++) {
            o.i(pop_n[i]);
            o.t(" ");
        }
    } else {
        o.t(" -t 5.0 ");
    }
    out += "\n1350154902\n\n";
}

// snp -o 2: print_ms (pop_snp.cpp:270-303) for one window [wbeg, wend): positions relative to
// the window as std::setprecision(8) (printf "%.8g"), then one 0/1 string per sample, the
// derived bit flipped where the outgroup carries it.
void format_ms_window(std::string &out, int n, uint32_t flag, int outidx, int32_t wbeg, int32_t wend,
                      const std::vector<int32_t> &pos, const std::vector<mask128> &types) {
    W o{out};
    const size_t S = pos.size();
    o.t("//\nsegsites: ");
    o.i((long long)S);
    o.t("\npositions: ");
    for (size_t i = 0; i < S; i++) {
        char b[64];
        std::snprintf(b, sizeof b, "%.8g ", (double)(unsigned)(pos[i] - wbeg) / (double)(wend - wbeg));
        out += b;
    }
    out += "\n";
    for (int i = 0; i < n; i++) {
        for (size_t j = 0; j < S; j++) {
            const bool d = (types[j] >> i) & 1;
            const bool flip = (flag & PBG_F_OUTGROUP) && ((types[j] >> outidx) & 1);
            out += d != flip ? '1' : '0';
        }
        out += "\n";
    }
    out += "\n";
}

}  // namespace pbg
