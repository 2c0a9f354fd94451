// format.cpp -- TSV writer, byte-identical to the reference's print_<stat> functions.
//
// The reference streams to std::cout with `std::fixed << std::setprecision(5)` (sticky),
// which libstdc++ renders through printf's "%.5f"; "NA" cells are `"\t" << std::setw(7) <<
// "NA"`, i.e. five spaces then NA.  Integers print in decimal.
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
void format_sweep_site(std::string &out, const pbg_cmd &c, int np, const uint64_t *pop_mask, uint32_t flag,
                       int32_t pos, uint64_t types) {
    W o{out};
    o.t(c.chr_name);
    o.t("\t");
    o.i((long long)pos + 1);
    for (int j = 0; j < np; j++) {
        const uint64_t pt = types & pop_mask[j];
        const unsigned pop_n = (unsigned)__builtin_popcountll(pop_mask[j]);
        const bool flip = (flag & PBG_F_OUTGROUP) && ((types >> c.outidx) & 1);
        const unsigned freq = (unsigned short)(flip ? pop_n - (unsigned)__builtin_popcountll(pt)
                                                    : (unsigned)__builtin_popcountll(pt));
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
                      const std::vector<int32_t> &pos, const std::vector<uint64_t> &types) {
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
