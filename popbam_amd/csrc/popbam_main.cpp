// popbam_main.cpp -- the native `popbam` host binary: the drop-in command line.
//
// "The build's popbam host binary does: subcommand CLI -> window planner -> host
// pileup feeder -> these exports -> TSV writer."  One process per command, as the reference:
//   main                  popbam.cpp:53-77 (argv[1] dispatch, "Error: unrecognized command")
//   parseCommandLine      GetOpt_pp (getopt_pp.cpp:68-147, getopt_pp.h:74-360): tokens, value
//                         options extracted in each command's order with std::stringstream
//                         conversion (so "-a 7" is 55 and "-a 20" is '2' = 50, Appendix A.12),
//                         OptionPresent flags, the free tokens as <in.bam> <region>
//   checkBAM              popbam.cpp:95-143 (BAM, -h header text, .bai, FASTA)
//   bam_smpl_add          pop_sample.cpp:15-107 (@RG ID/SM/PO), assign_pops popbam.cpp:145-171
//   bam_parse_region      pop_utils.cpp:386-461 (incl. "chr:a" = one base, A.13)
//   main_<cmd> loop       pop_nucdiv.cpp:37-125: here one walk of each block of whole windows
//                         (libpopbam_feed.so pbf_kstream_*: BGZF, pileup, per-sample partition and
//                         call_base's per-read loop on worker threads), every piece pushed to the
//                         GPU as it comes (libpopbam_gpu.so pbg_stream_*), then the window loop
//                         and print_<cmd> on the device / in format.cpp.
// The GPU context (HIP initialisation, cal_coef's tables, their upload) is built on a second
// thread while the main thread reads the FASTA contig and the feeder's workers start walking,
// so a fresh process pays the larger of the two, not their sum.
//
// Multi-GPU: POPBAM_WORLD=N forks N rank processes before anything touches the GPU; rank r
// computes its contiguous block of windows (the reference's own geometry with beg' / end',
// popbam_amd/shard.py) on device r mod (visible devices) and returns its text through a pipe;
// the parent prints the blocks in rank order (byte-identical to one GPU) or the first failing
// rank's error.  No collective: windows are independent.
//
// Errors are reported like fatal_error (pop_utils.cpp:510-519): "popbam runtime error:",
// the message, "Exiting program", exit status 1.  POPBAM_PROFILE=1 prints a JSON line of
// phase times to stderr (POPBAM_PROFILE=<path> writes it to that file).
#include <poll.h>
#include <sched.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/popbam_feed.h"
#include "../../include/popbam_gpu.h"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Fatal {
    std::string msg;
};

// BAM_* option bits (popbam.h:59-94)
enum : uint32_t {
    BAM_VARIANT = 0x01, BAM_ILLUMINA = 0x02, BAM_WINDOW = 0x04, BAM_MINPOPSAMPLE = 0x08, BAM_SUBSTITUTE = 0x10,
    BAM_HETEROZYGOTE = 0x20, BAM_OUTGROUP = 0x40, BAM_HEADERIN = 0x80
};

const char *kUsage =
    "\n"
    "Program: popbam (MI355X hot path: consensus call + window statistics on the GPU)\n"
    "\n"
    "Usage:   popbam <command> [options] <in.bam> <region>\n"
    "\n"
    "Command: snp         call SNPs\n"
    "         haplo       haplotype-based statistics\n"
    "         diverge     divergence from the reference\n"
    "         tree        neighbour-joining tree per window (pdist or jc)\n"
    "         nucdiv      nucleotide diversity (pi, dxy)\n"
    "         ld          linkage disequilibrium (ZnS, omega_max, Wall's B/Q)\n"
    "         sfs         site frequency spectrum (Tajima's D, Fay-Wu H)\n";

int cmd_id(const std::string &c) {   // pbg_cmd.cmd (include/popbam_gpu.h PBG_CMD_*)
    static const std::map<std::string, int> ids = {{"snp", PBG_CMD_SNP},       {"haplo", PBG_CMD_HAPLO},
                                                   {"diverge", PBG_CMD_DIVERGE}, {"tree", PBG_CMD_TREE},
                                                   {"nucdiv", PBG_CMD_NUCDIV},   {"ld", PBG_CMD_LD},
                                                   {"sfs", PBG_CMD_SFS}};
    auto it = ids.find(c);
    return it == ids.end() ? -1 : it->second;
}

// ---- parseCommandLine ------------------------------------------------------------------
struct Options {
    std::string cmd, reffile, headfile, bamfile, region, outgroup, dist = "pdist";
    uint32_t flag = 0;
    int min_depth = 3, max_depth = 255, min_rmsQ = 25, min_snpQ = 25;   // popbam.cpp:79-93
    unsigned char min_mapQ = 13, min_baseQ = 13;
    int min_sites = 10, output = 0, min_snps = 10, min_freq = 1;          // <cmd>Data constructors
    unsigned int win_size = 0;
    long double het_prior = 0.0001L;                                      // -z: parsed, unused
};

// GetOpt_pp token kinds (getopt_pp.h:45-58)
enum TokType { kGlobal, kUnknownYet, kPossibleNeg, kShort, kLong, kOptionArg, kGlobalUsed };
struct Tok {
    TokType t;
    std::string v;
};

// convert<T> (getopt_pp.h:133-144): stringstream extraction straight into the target; the
// target keeps whatever the extraction wrote even when the conversion is reported bad
template <class T> bool convert(const std::string &s, T &target) {
    std::stringstream ss;
    ss << s;
    ss >> target;
    return !(ss.fail() || !ss.eof());
}

struct Tokens {
    std::vector<Tok> toks;
    std::map<char, size_t> shortops;   // last occurrence wins
    bool any = false;

    void add(const std::string &a) {   // GetOpt_pp::_parse, getopt_pp.cpp:82-144
        if (a.size() > 1 && a[0] == '-') {
            if (a[1] == '-') {
                toks.push_back({a.size() > 2 ? kLong : kGlobal, a});
            } else {
                int i = 0;
                float f = 0.0f;
                if (convert(a, i)) {
                    if (a.size() > 2) {
                        toks.push_back({any ? kUnknownYet : kGlobal, a});
                    } else {
                        shortops[a[1]] = toks.size();
                        toks.push_back({kPossibleNeg, a});
                    }
                } else if (convert(a, f)) {
                    toks.push_back({any ? kUnknownYet : kGlobal, a});
                } else {
                    for (size_t j = 1; j < a.size(); ++j) {
                        shortops[a[j]] = toks.size();
                        toks.push_back({kShort, std::string(1, a[j])});
                    }
                }
            }
            any = true;
        } else if (a.size() > 1 && a[0] == '@') {   // options file (getopt_pp.cpp:53-66)
            std::ifstream in(a.substr(1));
            if (!in) throw Fatal{"options file " + a.substr(1) + " not found"};
            std::string w;
            while (in >> w) add(w);
        } else {
            toks.push_back({any ? kUnknownYet : kGlobal, a});
        }
    }
    // Option(letter, target): the token after the option's last occurrence, if it can be one
    template <class T> void value(char letter, T &target) {
        auto it = shortops.find(letter);
        if (it == shortops.end()) return;
        const size_t i = it->second + 1;
        if (i >= toks.size()) return;
        Tok &t = toks[i];
        if (t.t != kUnknownYet && t.t != kOptionArg && t.t != kPossibleNeg) return;   // NoArgs
        if (t.t == kPossibleNeg) shortops.erase(t.v[1]);
        t.t = kOptionArg;
        (void)convert(t.v, target);   // a bad conversion is ignored by every parseCommandLine
    }
    bool present(char letter) const { return shortops.count(letter) != 0; }
    std::vector<std::string> globals() const {
        std::vector<std::string> g;
        for (const Tok &t : toks)
            if (t.t == kGlobal || t.t == kUnknownYet || t.t == kPossibleNeg) g.push_back(t.v);
        return g;
    }
};

template <> bool convert<std::string>(const std::string &s, std::string &target) {
    target = s;
    return true;
}

// each command's parseCommandLine (pop_nucdiv.cpp:297-345, pop_sfs.cpp, pop_ld.cpp, pop_diverge.cpp,
// pop_haplo.cpp, pop_snp.cpp, pop_tree.cpp:590-612): value options in their extraction order,
// then the OptionPresent flags
Options parse_args(const std::string &cmd, const std::vector<std::string> &argv) {
    Options o;
    o.cmd = cmd;
    if (cmd == "diverge") o.win_size = 1;
    Tokens tk;
    for (const std::string &a : argv) tk.add(a);
    auto common = [&] {   // f h m x q: the first five extractions of every command but haplo
        tk.value('f', o.reffile);
        tk.value('h', o.headfile);
        tk.value('m', o.min_depth);
        tk.value('x', o.max_depth);
        tk.value('q', o.min_rmsQ);
    };
    if (cmd == "nucdiv") {
        common();
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('k', o.min_sites);
        tk.value('w', o.win_size);
    } else if (cmd == "sfs") {
        common();
        tk.value('p', o.outgroup);
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('k', o.min_sites);   // read, never used by sfs (A.12)
        tk.value('w', o.win_size);
    } else if (cmd == "ld") {
        common();
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('o', o.output);
        tk.value('z', o.het_prior);
        tk.value('n', o.min_snps);
        tk.value('w', o.win_size);
        tk.value('k', o.min_sites);
    } else if (cmd == "diverge") {
        common();
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('k', o.min_sites);
        tk.value('p', o.outgroup);
        tk.value('w', o.win_size);
        tk.value('o', o.output);
        tk.value('d', o.dist);
    } else if (cmd == "haplo") {
        tk.value('f', o.reffile);
        tk.value('h', o.headfile);
        tk.value('o', o.output);
        tk.value('m', o.min_depth);
        tk.value('x', o.max_depth);
        tk.value('q', o.min_rmsQ);
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('k', o.min_sites);
        tk.value('w', o.win_size);
    } else if (cmd == "snp") {
        common();
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('o', o.output);
        tk.value('z', o.het_prior);
        tk.value('p', o.outgroup);
        tk.value('w', o.win_size);
    } else if (cmd == "tree") {
        common();
        tk.value('s', o.min_snpQ);
        tk.value('a', o.min_mapQ);
        tk.value('b', o.min_baseQ);
        tk.value('k', o.min_sites);
        tk.value('w', o.win_size);
        tk.value('d', o.dist);
    } else {
        throw Fatal{"unrecognized command: " + cmd};
    }
    static const std::map<std::string, std::string> present_w = {
        {"nucdiv", "whpin"}, {"sfs", "whpi"}, {"ld", "whie"}, {"diverge", "whpnti"}, {"haplo", "whi"},
        {"snp", "whvizp"},   {"tree", "whi"}};
    const std::string &pw = present_w.at(cmd);
    auto asks = [&](char c) { return pw.find(c) != std::string::npos && tk.present(c); };
    if (asks('w')) {
        o.win_size *= 1000u;
        o.flag |= BAM_WINDOW;
    }
    if (tk.present('h')) o.flag |= BAM_HEADERIN;
    if ((cmd == "nucdiv" || cmd == "sfs" || cmd == "diverge" || cmd == "snp") && tk.present('p')) o.flag |= BAM_OUTGROUP;
    if (tk.present('i')) o.flag |= BAM_ILLUMINA;
    if ((cmd == "nucdiv" || cmd == "diverge") && tk.present('n')) o.flag |= BAM_MINPOPSAMPLE;
    if (cmd == "diverge" && tk.present('t')) o.flag |= BAM_SUBSTITUTE;
    if (cmd == "sfs" && std::find(argv.begin(), argv.end(), std::string("--theta")) != argv.end())
        o.output |= 1;   // extension: S, theta_W and the spectrum after the reference's columns
    if (cmd == "ld" && tk.present('e')) o.min_freq = 2;
    if (cmd == "snp" && tk.present('v')) o.flag |= BAM_VARIANT;
    if (cmd == "snp" && tk.present('z')) o.flag |= BAM_HETEROZYGOTE;
    if ((cmd == "diverge" || cmd == "tree") && o.dist != "pdist" && o.dist != "jc")
        throw Fatal{o.dist + " is not a valid distance option"};
    if ((cmd == "ld" || cmd == "haplo" || cmd == "snp") && (o.output < 0 || o.output > 2))
        throw Fatal{"Not a valid output option"};
    if (cmd == "diverge" && (o.output < 0 || o.output > 1)) throw Fatal{"Not a valid output option"};
    const std::vector<std::string> g = tk.globals();
    if (g.size() < 2) throw Fatal{"Need to specify BAM file name"};
    o.bamfile = g[0];
    o.region = g[1];
    return o;
}

// ---- bam_smpl_add / assign_pops -------------------------------------------------------
struct SampleModel {
    std::vector<std::string> samples, pops;
    std::vector<std::string> rg_ids;
    std::vector<int32_t> rg_sample;
    std::vector<int> sample_pop;
};

int index_of(const std::vector<std::string> &v, const std::string &s) {
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == s) return (int)i;
    return -1;
}

// pop_sample.cpp:15-107: after each "@RG" the next "\tID:", "\tSM:" and "\tPO:" anywhere in the
// text; the first sample / population name seen gets the next index
SampleModel parse_header(const std::string &text, const std::string &bamfile) {
    SampleModel m;
    std::map<std::string, int> spop;
    auto field = [&](size_t i) {
        size_t j = i;
        while (j < text.size() && text[j] != '\t' && text[j] != '\n') ++j;
        return text.substr(i, j - i);
    };
    size_t p = 0;
    int n = 0;
    for (;;) {
        const size_t q = text.find("@RG", p);
        if (q == std::string::npos) break;
        p = q + 3;
        size_t qi = text.find("\tID:", p), ri = text.find("\tSM:", p), si = text.find("\tPO:", p);
        const long QI = qi == std::string::npos ? -1 : (long)qi + 4, RI = ri == std::string::npos ? -1 : (long)ri + 4,
                   SI = si == std::string::npos ? -1 : (long)si + 4;
        if (RI < 0 || QI < 0) break;
        const std::string rg = field(QI), sm = field(RI);
        if (index_of(m.rg_ids, rg) < 0) {
            if (index_of(m.samples, sm) < 0) m.samples.push_back(sm);
            m.rg_ids.push_back(rg);
            m.rg_sample.push_back(index_of(m.samples, sm));
        }
        if (SI >= 0) {
            const std::string po = field(SI);
            if (!spop.count(sm)) {
                if (index_of(m.pops, po) < 0) m.pops.push_back(po);
                spop[sm] = index_of(m.pops, po);
            }
        }
        p = (size_t)std::max({QI, RI, SI});
        ++n;
    }
    if (n == 0) {   // no @RG: one sample and population named after the file
        m.samples = {bamfile};
        m.pops = {bamfile};
        spop[bamfile] = 0;
    }
    for (const std::string &s : m.samples) {
        auto it = spop.find(s);
        if (it == spop.end())
            throw Fatal{"Sample " + s + " not assigned to a population.\nPlease check BAM header file definitions"};
        m.sample_pop.push_back(it->second);
    }
    return m;
}

// get_refid (pop_utils.cpp:463-498): the first "AS:" value, up to a tab or newline
std::string get_refid(const std::string &text) {
    const size_t v = text.find("AS:");
    if (v == std::string::npos)
        throw Fatal{"Unable to parse reference sequence name\nBe sure the AS tag is defined in the sequence dictionary"};
    size_t w = v + 3;
    while (w < text.size() && text[w] != '\t' && text[w] != '\n') ++w;
    return text.substr(v + 3, std::min<size_t>(w - (v + 3), 199));
}

long atoi_prefix(const std::string &s) {   // atoi: leading integer, 0 when none
    size_t i = 0;
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    size_t j = i;
    if (j < s.size() && (s[j] == '+' || s[j] == '-')) ++j;
    const size_t d = j;
    while (j < s.size() && std::isdigit((unsigned char)s[j])) ++j;
    if (j == d) return 0;
    return std::strtol(s.substr(i, j - i).c_str(), nullptr, 10);
}

// bam_parse_region (pop_utils.cpp:386-461) -> (tid, beg, end)
void parse_region(const std::string &region, const std::vector<std::string> &names, const std::vector<int64_t> &lengths,
                  int &tid, int &beg, int &end) {
    std::string r;
    for (char ch : region)
        if (ch != ' ' && ch != ',') r += ch;
    const size_t l = r.size();
    size_t name_end = r.find(':');
    if (name_end == std::string::npos) name_end = l;
    std::string nm;
    if (name_end < l) {
        const std::string coords = r.substr(name_end + 1);
        bool bad = std::count(coords.begin(), coords.end(), '-') > 1;
        for (char ch : coords) bad = bad || !(std::isdigit((unsigned char)ch) || ch == ',' || ch == '-');
        if (bad) name_end = l;
        nm = r.substr(0, name_end);
        if (index_of(names, nm) < 0) {
            if (index_of(names, r) < 0) throw Fatal{"Bad genome coordinates: " + region};
            nm = r;
        }
    } else {
        nm = r;
        if (index_of(names, nm) < 0) throw Fatal{"Bad genome coordinates: " + region};
    }
    tid = index_of(names, nm);
    if (name_end < l) {
        const std::string coords = r.substr(name_end + 1);
        const size_t dash = coords.find('-');
        const std::string first = dash == std::string::npos ? coords : coords.substr(0, dash);
        const std::string last = dash == std::string::npos ? coords : coords.substr(dash + 1);
        long b = atoi_prefix(first);
        if (b > 0) --b;
        beg = (int)b;
        end = (int)atoi_prefix(last);
    } else {
        beg = 0;
        end = (int)lengths[tid];
    }
    if (beg > end) throw Fatal{"Bad genome coordinates: " + region};
}

// ---- window geometry (popbam_amd/shard.py) -----------------------------------------------
int64_t num_windows(int64_t beg, int64_t end, int64_t w, bool windowed) {
    if (!windowed) return 1;
    return std::max<int64_t>(0, ((end - beg) - 1) / w);
}

bool shard_region(int64_t beg, int64_t end, int64_t w, bool windowed, int rank, int world, int64_t &b2, int64_t &e2) {
    if (!windowed) {
        b2 = beg, e2 = end;
        return rank == 0;
    }
    const int64_t nw = num_windows(beg, end, w, true), q = nw / world, r = nw % world;
    const int64_t a = rank * q + std::min<int64_t>(rank, r), b = a + q + (rank < r ? 1 : 0);
    if (a == b) return false;
    b2 = beg + a * w, e2 = beg + b * w + 1;
    return true;
}

void positions_needed(int64_t beg, int64_t end, int64_t w, bool windowed, int64_t &lo, int64_t &hi) {
    if (!windowed) {
        lo = beg, hi = end;
        return;
    }
    const int64_t nw = num_windows(beg, end, w, true);
    lo = beg;
    hi = nw ? beg + nw * w - 1 : beg;
}

// blocks of whole windows of about block_sites positions (cli.window_blocks)
std::vector<std::pair<int64_t, int64_t>> window_blocks(int64_t beg, int64_t end, int64_t w, bool windowed,
                                                       int64_t block_sites) {
    if (!windowed) return {{beg, end}};
    const int64_t nw = num_windows(beg, end, w, true), per = std::max<int64_t>(1, block_sites / std::max<int64_t>(1, w));
    std::vector<std::pair<int64_t, int64_t>> out;
    for (int64_t a = 0; a < nw; a += per) out.push_back({beg + a * w, beg + std::min(nw, a + per) * w + 1});
    return out;
}

// ---- phase profile -------------------------------------------------------------------
struct Profile {
    std::vector<std::pair<std::string, double>> t;
    pbf_profile feed{};
    pbg_stream_prof gpu{};
    int threads = 0, piece = 0, blocks = 0;
    void add(const std::string &k, double v) {
        for (auto &e : t)
            if (e.first == k) {
                e.second += v;
                return;
            }
        t.push_back({k, v});
    }
    std::string json() const {
        std::ostringstream s;
        s.precision(6);
        s << "{\"popbam_profile\": {";
        for (auto &e : t) s << "\"" << e.first << "\": " << std::fixed << e.second << ", ";
        s << "\"feeder_threads\": " << threads << ", \"piece_sites\": " << piece << ", \"blocks\": " << blocks
          << ", \"feeder\": {\"t_wall\": " << feed.t_wall << ", \"t_fetch\": " << feed.t_fetch
          << ", \"t_inflate\": " << feed.t_inflate << ", \"t_walk\": " << feed.t_walk
          << ", \"t_consumer_wait\": " << feed.t_consumer_wait << ", \"records\": " << feed.records
          << ", \"pieces\": " << feed.pieces << "}, \"gpu\": {\"h2d_bytes\": " << gpu.h2d_bytes
          << ", \"chunks\": " << gpu.chunks << ", \"ms_stage\": " << gpu.ms_stage << ", \"ms_wait\": " << gpu.ms_wait
          << ", \"ms_h2d\": " << gpu.ms_h2d << ", \"ms_call\": " << gpu.ms_call << ", \"ms_finish\": " << gpu.ms_finish
          << "}}}";
        return s.str();
    }
};

// the process's own start (from /proc/self/stat, clock ticks after boot) to now, in seconds:
// exec + dynamic loading of the libraries before main
double since_process_start() {
    std::ifstream f("/proc/self/stat");
    std::string s;
    std::getline(f, s);
    const size_t rp = s.rfind(')');
    if (rp == std::string::npos) return -1.0;
    std::istringstream in(s.substr(rp + 2));
    std::string tok;
    unsigned long long start = 0;
    for (int field = 3; in >> tok; ++field)
        if (field == 22) {
            start = std::strtoull(tok.c_str(), nullptr, 10);
            break;
        }
    std::ifstream up("/proc/uptime");
    double uptime = 0.0;
    up >> uptime;
    const double hz = (double)sysconf(_SC_CLK_TCK);
    return start ? uptime - (double)start / hz : -1.0;
}

int host_cores() {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) return std::max(1, CPU_COUNT(&cs));
    return std::max(1u, std::thread::hardware_concurrency());
}

int env_int(const char *name, long dflt) {
    const char *v = std::getenv(name);
    return v && *v ? (int)std::strtol(v, nullptr, 10) : (int)dflt;
}

// ---- pieces are freed on a thread of their own ---------------------------------------------
// A piece's arrays are tens of MB (munmap + TLB shootdowns across the feeder's threads: ~1.4 ms
// each, ~0.1 s per 5 Mbp command on the main thread); the process ends right after its run, so
// whatever is still queued then goes with it.
struct Freer {
    std::mutex m;
    std::condition_variable cv;
    std::vector<pbf_keys> q;
    bool stop = false;
    std::thread th;
    Freer() {
        th = std::thread([this] {
            std::unique_lock<std::mutex> lk(m);
            for (;;) {
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                std::vector<pbf_keys> batch;
                batch.swap(q);
                lk.unlock();
                for (auto &p : batch) pbf_keys_free(&p);
                lk.lock();
            }
        });
    }
    void put(const pbf_keys &p) {
        {
            std::lock_guard<std::mutex> lk(m);
            q.push_back(p);
        }
        cv.notify_one();
    }
    ~Freer() {   // normal teardown (errors, POPBAM_DESTROY): drain and join
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_one();
        th.join();
    }
};

Freer *freer() {   // one per process, never destroyed (see above)
    static Freer *f = new Freer();
    return f;
}

// ---- the GPU context, built on its own thread -------------------------------------------
struct GpuInit {
    std::thread th;
    std::atomic<bool> done{false};
    pbg_params P{};
    int device = 0, rc = PBG_OK;
    pbg_ctx *ctx = nullptr;
    std::string err;
    double t_hip_init = 0.0, t_create = 0.0;
    bool started = false;

    void start() {
        started = true;
        th = std::thread([this] {
            const auto t0 = Clock::now();
            (void)pbg_device_count();   // HIP runtime initialisation, timed on its own
            const auto t1 = Clock::now();
            rc = pbg_create(&ctx, device, &P);
            if (rc != PBG_OK) err = pbg_last_error(nullptr);
            t_hip_init = secs(t0, t1);
            t_create = secs(t1, Clock::now());
            done.store(true);
        });
    }
    void join() {
        if (started && th.joinable()) th.join();
    }
    ~GpuInit() { join(); }
};

std::string read_file(const std::string &path) {
    std::ifstream in(path, std::ios::binary);
    std::ostringstream s;
    s << in.rdbuf();
    return s.str();
}

bool file_exists(const std::string &p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0;
}

// One `popbam <cmd> argv...` (rank `rank` of `world`: only this rank's block of windows).
std::string run(const std::string &cmd, const std::vector<std::string> &argv, int device, int rank, int world,
                Profile &prof) {
    const auto t_start = Clock::now();
    Options o = parse_args(cmd, argv);
    if (!file_exists(o.bamfile)) throw Fatal{"Cannot read BAM file " + o.bamfile};
    pbf_bam *bam = nullptr;
    if (pbf_open(&bam, o.bamfile.c_str()) < 0) throw Fatal{"Cannot read BAM file " + o.bamfile + ": " + pbf_last_error()};
    struct BamCloser {
        pbf_bam *b;
        ~BamCloser() { pbf_close(b); }
    } bam_closer{bam};
    std::string header = pbf_header_text(bam);
    if (o.flag & BAM_HEADERIN) header = read_file(o.headfile);
    if (!pbf_has_index(bam)) throw Fatal{"Index file not available for BAM file " + o.bamfile};
    if (o.reffile.empty() || !file_exists(o.reffile))
        throw Fatal{"Failed to load index for fastA reference file: " + o.reffile};
    const SampleModel sm = parse_header(header, o.bamfile);
    const int n = (int)sm.samples.size(), npops = (int)sm.pops.size();
    int outidx = 0;   // sfs / diverge / snp check -p right after bam_smpl_add (pop_sfs.cpp:37-50,
                      // pop_diverge.cpp:37-50, pop_snp.cpp:36-49): the last sample of that name
    if ((o.flag & BAM_OUTGROUP) && (cmd == "sfs" || cmd == "diverge" || cmd == "snp")) {
        int found = -1;
        for (int i = 0; i < n; ++i)
            if (sm.samples[i] == o.outgroup) found = i;
        if (found < 0) throw Fatal{"Specified outgroup " + o.outgroup + " not found"};
        outidx = found;
    }
    // pbg_params (engine.make_params): checked now, reported where the reference order puts them
    std::string param_err;
    if (o.max_depth < 0) param_err = "maximum read depth -x " + std::to_string(o.max_depth) + " must not be negative";
    else if (npops > PBG_MAX_POPS) param_err = "more than " + std::to_string(PBG_MAX_POPS) + " populations";
    else if (n > PBG_MAX_SAMPLES) param_err = "more than " + std::to_string(PBG_MAX_SAMPLES) + " samples";
    const int max_depth = std::min(o.max_depth, 65535);   // the pileup holds at most 8000 reads
    GpuInit gi;
    gi.device = device;
    if (param_err.empty()) {
        pbg_params &P = gi.P;
        P.n_samples = n;
        P.n_pops = npops;
        for (int v = 0; v < n; ++v) {
            const int p = sm.sample_pop[v];
            if (v < 64) P.pop_mask[p] |= 1ull << v;
            else P.pop_mask_hi[p] |= 1ull << (v - 64);
            P.pop_n[p]++;
        }
        P.min_depth = o.min_depth;
        P.max_depth = max_depth;
        P.min_rmsQ = o.min_rmsQ;
        P.min_snpQ = o.min_snpQ;
        P.min_mapQ = o.min_mapQ;
        P.min_baseQ = o.min_baseQ;
        P.flag = o.flag;
        gi.start();   // HIP init + cal_coef + upload while the host reads and walks
    }
    prof.add("parse_s", secs(t_start, Clock::now()));
    const std::string refid = cmd == "tree" ? get_refid(header) : std::string();
    std::vector<std::string> names;
    std::vector<int64_t> lengths;
    for (int i = 0; i < pbf_n_refs(bam); ++i) {
        names.push_back(pbf_ref_name(bam, i));
        lengths.push_back(pbf_ref_len(bam, i));
    }
    int tid = 0, beg = 0, end = 0;
    parse_region(o.region, names, lengths, tid, beg, end);
    auto t0 = Clock::now();
    char *seqp = nullptr;
    int64_t seqlen = 0;
    if (pbf_fasta_fetch(o.reffile.c_str(), names[tid].c_str(), &seqp, &seqlen) < 0)
        throw Fatal{"Failed to load index for fastA reference file: " + o.reffile + ": " + pbf_last_error()};
    std::string seq(seqp, (size_t)seqlen);
    pbf_free(seqp);
    if ((int64_t)seq.size() < end) seq.append((size_t)end - seq.size(), 'N');   // no reference base
    prof.add("fasta_s", secs(t0, Clock::now()));
    const bool windowed = (o.flag & BAM_WINDOW) != 0;
    const int threads = env_int("POPBAM_FEED_THREADS", std::min(16, host_cores()));
    const int piece = env_int("POPBAM_FEED_CHUNK", 1 << 16);
    prof.threads = threads, prof.piece = piece;
    const int64_t nw_total = num_windows(beg, end, o.win_size, windowed);
    int64_t rbeg = beg, rend = end, ms0 = nw_total;
    if (world > 1) {
        if (!shard_region(beg, end, o.win_size, windowed, rank, world, rbeg, rend)) return std::string();
        ms0 = rank == 0 ? nw_total : -1;
    }
    // consensus words (snp -o 0) cost n * 8 bytes per position on the device and the host:
    // blocks of at most ~1 GB of them
    int64_t block_sites = env_int("POPBAM_BLOCK_SITES", 1 << 26);
    if (cmd == "snp" && o.output == 0) block_sites = std::min<int64_t>(block_sites, std::max<int64_t>(1 << 16, (1ll << 30) / (8ll * n)));
    const auto blocks = window_blocks(rbeg, rend, o.win_size, windowed, block_sites);
    if (blocks.empty()) return std::string();
    if (!param_err.empty()) throw Fatal{param_err};
    // compact pieces (pbg_stream_push_compact: the reference-only tasks' keys stay on the host)
    // for every command but snp -o 0, whose consensus words need every task's keys;
    // POPBAM_COMPACT=0 pushes the full pieces
    const bool compact = !(cmd == "snp" && o.output == 0) && max_depth <= 33025 && env_int("POPBAM_COMPACT", 1) != 0;
    const pbf_filter flt{o.min_baseQ, o.min_mapQ, (o.flag & BAM_ILLUMINA) ? 1 : 0, max_depth <= 255 ? 1 : 2,
                         compact ? 1 : 0};
    std::vector<const char *> sn, pn, rg;
    for (auto &s : sm.samples) sn.push_back(s.c_str());
    for (auto &s : sm.pops) pn.push_back(s.c_str());
    for (auto &s : sm.rg_ids) rg.push_back(s.c_str());
    const int32_t fallback = sm.rg_ids.empty() ? 0 : -1;
    std::string text;
    pbg_ctx *ctx = nullptr;
    for (size_t bi = 0; bi < blocks.size(); ++bi) {
        const int64_t b0 = blocks[bi].first, b1 = blocks[bi].second;
        int64_t lo, hi;
        positions_needed(b0, b1, o.win_size, windowed, lo, hi);
        hi = std::max(hi, lo);
        pbg_cmd c{};
        c.cmd = cmd_id(cmd);
        c.output = o.output;
        c.min_sites = o.min_sites;
        c.min_snps = o.min_snps;
        c.min_freq = o.min_freq;
        c.outidx = outidx;
        c.jc = o.dist == "jc" ? 1 : 0;
        c.windowed = windowed ? 1 : 0;
        c.win_size = o.win_size;
        c.beg = (int32_t)b0;
        c.end = (int32_t)b1;
        c.chr_name = names[tid].c_str();
        c.sample_names = sn.data();
        c.pop_names = pn.data();
        c.refid = refid.c_str();
        c.ms_windows = (blocks.size() > 1 || world > 1) ? (int32_t)(bi == 0 ? ms0 : -1) : 0;
        t0 = Clock::now();
        pbf_kstream *ks = nullptr;
        if (pbf_kstream_open(o.bamfile.c_str(), std::max(1, threads), piece, tid, (int32_t)lo, (int32_t)hi,
                             windowed ? (int32_t)o.win_size : 0, seq.c_str(), rg.data(), sm.rg_sample.data(),
                             (int)rg.size(), fallback, n, max_depth, &flt, &ks) < 0)
            throw Fatal{"Failed to retrieve region " + o.region + ": " + pbf_last_error()};
        struct KsCloser {
            pbf_kstream *k;
            ~KsCloser() { pbf_kstream_close(k); }
        } ks_closer{ks};
        prof.add("kstream_open_s", secs(t0, Clock::now()));
        // Until the context thread is done (HIP init + tables), take the walk's pieces as they come
        // (up to ~3 GB), so the feeder's workers never stall on their look-ahead: the walk of a
        // fresh process's first block overlaps the GPU's initialisation instead of following it
        std::vector<pbf_keys> early;
        bool walked = false;
        struct EarlyFree {
            std::vector<pbf_keys> &v;
            ~EarlyFree() {
                for (auto &p : v) pbf_keys_free(&p);
            }
        } early_free{early};
        if (!ctx) {
            t0 = Clock::now();
            size_t held = 0;
            while (!gi.done.load() && held < (3ull << 30)) {
                pbf_keys p{};
                const int r = pbf_kstream_next(ks, &p);
                if (r < 0) {
                    if (r == PBF_E_RG) throw Fatal{"Problem assigning read group"};
                    throw Fatal{"Failed to retrieve region " + o.region + ": " + pbf_last_error()};
                }
                if (r == 0) {
                    walked = true;
                    break;
                }
                held += (size_t)p.n_sites * (1 + (size_t)n * (flt.k_bytes + 4)) + p.n_keys * 2;
                early.push_back(p);
            }
            prof.add("walk_during_gpu_init_s", secs(t0, Clock::now()));
            prof.add("pieces_during_gpu_init", (double)early.size());
        }
        if (!ctx) {   // the context thread: HIP init + tables
            t0 = Clock::now();
            gi.join();
            prof.add("gpu_join_wait_s", secs(t0, Clock::now()));
            prof.add("hip_init_s", gi.t_hip_init);
            prof.add("pbg_create_s", gi.t_create);
            if (gi.rc != PBG_OK) throw Fatal{"pbg_create failed (" + std::to_string(gi.rc) + "): " + gi.err};
            ctx = gi.ctx;
        }
        t0 = Clock::now();
        pbg_stream *st = nullptr;
        if (pbg_stream_open(ctx, &c, 1, (int32_t)lo, (uint32_t)(hi - lo), 0, &st) != PBG_OK)
            throw Fatal{std::string("pbg_stream_open failed: ") + pbg_last_error(ctx)};
        struct StCloser {
            pbg_stream *s;
            ~StCloser() { pbg_stream_close(s); }
        } st_closer{st};
        prof.add("stream_open_s", secs(t0, Clock::now()));
        t0 = Clock::now();
        bool first = true;
        // POPBAM_FAULT_PUSH=k (tests only): the k-th push of the run reports a failure, so the error
        // path -- pieces already handed to the freer, the rest still owned here -- is exercised
        const long fault_at = env_int("POPBAM_FAULT_PUSH", 0);
        long pushes = 0;
        auto push = [&](const pbg_pileup &pl) {
            if (++pushes == fault_at) return (int)PBG_E_BATCH;
            return compact ? pbg_stream_push_compact(st, &pl) : pbg_stream_push(st, &pl);
        };
        for (pbf_keys &p : early) {
            const auto tp = Clock::now();
            pbg_pileup pl{p.n_sites, p.pos0, p.ref, p.k, p.rmsq, p.block_off, p.keys};
            const int pr = push(pl);
            const auto tf = Clock::now();
            freer()->put(p);
            p = pbf_keys{};   // owned by the freer now: EarlyFree must not free it again on a throw
            prof.add("push_calls_s", secs(tp, tf));
            prof.add("keys_free_s", secs(tf, Clock::now()));
            if (pr != PBG_OK) throw Fatal{std::string("pbg_stream_push failed: ") + pbg_last_error(ctx)};
            if (first) prof.add("first_push_s", secs(tp, Clock::now()));
            first = false;
        }
        prof.add("push_early_s", secs(t0, Clock::now()));
        early.clear();
        while (!walked) {
            pbf_keys p{};
            const int r = pbf_kstream_next(ks, &p);
            if (r < 0) {
                if (r == PBF_E_RG) throw Fatal{"Problem assigning read group"};
                throw Fatal{"Failed to retrieve region " + o.region + ": " + pbf_last_error()};
            }
            if (r == 0) {
                walked = true;
                break;
            }
            pbg_pileup pl{p.n_sites, p.pos0, p.ref, p.k, p.rmsq, p.block_off, p.keys};
            const int pr = push(pl);
            freer()->put(p);
            if (pr != PBG_OK) throw Fatal{std::string("pbg_stream_push failed: ") + pbg_last_error(ctx)};
        }
        prof.add("walk_push_s", secs(t0, Clock::now()));
        t0 = Clock::now();
        if (pbg_stream_finish(st) != PBG_OK) throw Fatal{std::string("pbg_stream_finish failed: ") + pbg_last_error(ctx)};
        size_t need = 0;
        (void)pbg_stream_text(st, 0, nullptr, 0, &need);
        std::string part(need, '\0');
        const long len = pbg_stream_text(st, 0, &part[0], part.size(), &need);
        if (len < 0) throw Fatal{std::string("pbg_stream_text failed: ") + pbg_last_error(ctx)};
        part.resize((size_t)len);
        text += part;
        prof.add("finish_s", secs(t0, Clock::now()));
        pbf_profile fp{};
        if (pbf_kstream_profile(ks, &fp) == 0) {
            prof.feed.t_wall += fp.t_wall, prof.feed.t_fetch += fp.t_fetch, prof.feed.t_inflate += fp.t_inflate;
            prof.feed.t_walk += fp.t_walk, prof.feed.t_consumer_wait += fp.t_consumer_wait;
            prof.feed.records += fp.records, prof.feed.pieces += fp.pieces;
        }
        pbg_stream_prof gp{};
        if (pbg_stream_profile(st, &gp) == 0) {
            prof.gpu.h2d_bytes += gp.h2d_bytes, prof.gpu.chunks += gp.chunks, prof.gpu.ms_stage += gp.ms_stage;
            prof.gpu.ms_wait += gp.ms_wait, prof.gpu.ms_h2d += gp.ms_h2d, prof.gpu.ms_call += gp.ms_call;
            prof.gpu.ms_finish += gp.ms_finish;
        }
        ++prof.blocks;
    }
    prof.add("run_s", secs(t_start, Clock::now()));
    // the process ends right after this run (main exits with _exit): every stream has finished and
    // been closed, so nothing is in flight, and the context's device memory goes with the process
    // (pbg_destroy and the HIP runtime's teardown cost a fresh process ~0.15 s).  POPBAM_DESTROY=1
    // destroys it here all the same.
    if (ctx && env_int("POPBAM_DESTROY", 0)) pbg_destroy(ctx);
    return text;
}

void fatal_text(const std::string &msg) {
    std::string s = "popbam runtime error:\n" + msg + "\nExiting program\n";
    (void)!write(2, s.data(), s.size());
}

void emit_profile(const Profile &prof) {
    const char *p = std::getenv("POPBAM_PROFILE");
    if (!p || !*p || !std::strcmp(p, "0")) return;
    const std::string j = prof.json() + "\n";
    if (!std::strcmp(p, "1")) {
        (void)!write(2, j.data(), j.size());
    } else {
        std::ofstream f(p, std::ios::app);
        f << j;
    }
}

bool write_all(int fd, const char *p, size_t n) {
    while (n) {
        const ssize_t w = ::write(fd, p, n);
        if (w <= 0) return false;
        p += w, n -= (size_t)w;
    }
    return true;
}

// POPBAM_WORLD=N: fork N ranks before any HIP call; each writes "<status byte><text>" to a pipe
int run_ranks(int world, const std::string &cmd, const std::vector<std::string> &argv) {
    std::vector<pid_t> pids(world, -1);
    std::vector<int> fds(world, -1);
    std::fflush(stdout);
    std::fflush(stderr);
    for (int r = 0; r < world; ++r) {
        int pfd[2];
        if (pipe(pfd) != 0) {
            fatal_text("pipe failed");
            return 1;
        }
        const pid_t pid = fork();
        if (pid < 0) {
            fatal_text("fork failed");
            return 1;
        }
        if (pid == 0) {
            ::close(pfd[0]);
            for (int q = 0; q < r; ++q) ::close(fds[q]);
            Profile prof;
            std::string out;
            char status = 0;
            try {
                int ndev = pbg_device_count();
                const int dev = env_int("POPBAM_DEVICE", ndev > 0 ? r % ndev : 0);
                out = run(cmd, argv, dev, r, world, prof);
            } catch (const Fatal &f) {
                status = 1;
                out = f.msg;
            }
            emit_profile(prof);
            const bool ok = write_all(pfd[1], &status, 1) && write_all(pfd[1], out.data(), out.size());
            ::close(pfd[1]);
            std::fflush(nullptr);
            _exit(ok ? 0 : 1);
        }
        ::close(pfd[1]);
        pids[r] = pid, fds[r] = pfd[0];
    }
    // read every rank's pipe as it fills (a rank blocks on a full pipe otherwise)
    std::vector<std::string> got(world);
    std::vector<bool> open(world, true);
    int left = world;
    while (left) {
        std::vector<pollfd> pf;
        std::vector<int> who;
        for (int r = 0; r < world; ++r)
            if (open[r]) pf.push_back({fds[r], POLLIN, 0}), who.push_back(r);
        if (poll(pf.data(), pf.size(), -1) < 0) break;
        for (size_t i = 0; i < pf.size(); ++i) {
            if (!(pf[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
            char buf[1 << 16];
            const ssize_t k = ::read(pf[i].fd, buf, sizeof buf);
            if (k > 0) {
                got[who[i]].append(buf, (size_t)k);
            } else {
                ::close(pf[i].fd);
                open[who[i]] = false;
                --left;
            }
        }
    }
    int worst = 0;
    for (int r = 0; r < world; ++r) {
        int stv = 0;
        (void)waitpid(pids[r], &stv, 0);
        if (!WIFEXITED(stv) || WEXITSTATUS(stv) != 0) worst = 1;
    }
    for (int r = 0; r < world; ++r) {   // the first failing rank's message, in rank order
        if (got[r].empty()) {
            fatal_text("rank " + std::to_string(r) + " ended without a result");
            return 1;
        }
        if (got[r][0] != 0) {
            fatal_text(got[r].substr(1));
            return 1;
        }
    }
    if (worst) {
        fatal_text("a rank process failed");
        return 1;
    }
    for (int r = 0; r < world; ++r)
        if (!write_all(1, got[r].data() + 1, got[r].size() - 1)) return 1;
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fputs(kUsage, stderr);
        return 1;
    }
    const std::string cmd = argv[1];
    if (cmd_id(cmd) < 0) {
        std::fprintf(stderr, "Error: unrecognized command: %s\n", argv[1]);
        return 1;
    }
    const std::vector<std::string> args(argv + 2, argv + argc);
    const int world = env_int("POPBAM_WORLD", 1);
    if (world > 1) return run_ranks(world, cmd, args);
    if (env_int("WORLD_SIZE", 1) > 1) {
        fatal_text("torchrun launches run `python -m popbam_amd.cli`; the native binary shards with POPBAM_WORLD=N");
        return 1;
    }
    Profile prof;
    prof.add("process_start_to_main_s", since_process_start());
    prof.add("main_wall_epoch_s", std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
    std::string text;
    try {
        text = run(cmd, args, env_int("POPBAM_DEVICE", 0), 0, 1, prof);
    } catch (const Fatal &f) {
        fatal_text(f.msg);
        emit_profile(prof);
        std::fflush(nullptr);
        _exit(1);
    }
    const auto t0 = Clock::now();
    const bool ok = write_all(1, text.data(), text.size());
    prof.add("write_s", secs(t0, Clock::now()));
    prof.add("exit_wall_epoch_s", std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count());
    emit_profile(prof);
    std::fflush(nullptr);
    _exit(ok ? 0 : 1);   // see run(): no teardown of the device context / HIP runtime at exit
}
