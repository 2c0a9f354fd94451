"""Host-side mirror of POPBAM's command line, header and region handling.

Restates, for the subcommands on the hot path (snp, nucdiv, sfs, ld, diverge, haplo):
  * option parsing through GetOpt_pp (getopt_pp.cpp:66-140, getopt_pp.h:133-144, 200-360):
    a token after a value option is consumed as its argument; `OptionPresent` consumes
    nothing; the remaining free tokens are the globals (<in.bam> <region>).  Values are
    converted with `stringstream >> T`: an `unsigned char` option keeps the FIRST CHARACTER's
    code ("-a 7" -> 55; "-a 20" -> '2' = 50, reported as a parse error that the caller
    ignores), an int keeps the leading integer;
  * per-subcommand defaults (popbam.cpp:79-93 and each <cmd>Data constructor);
  * bam_parse_region (pop_utils.cpp:386-461) incl. the "chr:a" single-base form (A.13);
  * the sample / population model from @RG ID/SM/PO (pop_sample.cpp:15-107,
    popbam.cpp:145-171).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

# BAM_* option bits (popbam.h:59-94)
BAM_VARIANT = 0x01
BAM_ILLUMINA = 0x02
BAM_WINDOW = 0x04
BAM_MINPOPSAMPLE = 0x08
BAM_SUBSTITUTE = 0x10
BAM_HETEROZYGOTE = 0x20
BAM_OUTGROUP = 0x40
BAM_HEADERIN = 0x80

# popbam_func_t (popbam.h:208)
CMD_IDS = {"snp": 0, "haplo": 1, "diverge": 2, "tree": 3, "nucdiv": 4, "ld": 5, "sfs": 6}


class PopbamError(RuntimeError):
    """Mirrors fatal_error (pop_utils.cpp:510-519): message + non-zero exit in the CLI."""


@dataclass
class Options:
    cmd: str
    reffile: str = ""
    headfile: str = ""
    bamfile: str = ""
    region: str = ""
    flag: int = 0
    min_depth: int = 3
    max_depth: int = 255
    min_rmsQ: int = 25
    min_snpQ: int = 25
    min_mapQ: int = 13
    min_baseQ: int = 13
    min_sites: int = 10
    win_size: int = 0
    output: int = 0
    min_snps: int = 10
    min_freq: int = 1
    outgroup: str = ""
    dist: str = "pdist"
    errors: list = field(default_factory=list)


# which letters take a value, per subcommand, in the order parseCommandLine extracts them,
# with the conversion type: 's' string, 'i' int, 'u' unsigned int, 'c' unsigned char,
# 'L' long double
_VALUE_OPTS = {
    "nucdiv": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"), ("a", "c"),
               ("b", "c"), ("k", "i"), ("w", "u")],
    "sfs": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("p", "s"), ("s", "i"),
            ("a", "c"), ("b", "c"), ("k", "i"), ("w", "u")],
    "ld": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"), ("a", "c"),
           ("b", "c"), ("o", "i"), ("z", "L"), ("n", "i"), ("w", "u"), ("k", "i")],
    "diverge": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"), ("a", "c"),
                ("b", "c"), ("k", "i"), ("p", "s"), ("w", "u"), ("o", "i"), ("d", "s")],
    "haplo": [("f", "s"), ("h", "s"), ("o", "i"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"),
              ("a", "c"), ("b", "c"), ("k", "i"), ("w", "u")],
    "snp": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"), ("a", "c"),
            ("b", "c"), ("o", "i"), ("z", "L"), ("p", "s"), ("w", "u")],
    # treeData::parseCommandLine pop_tree.cpp:590-612
    "tree": [("f", "s"), ("h", "s"), ("m", "i"), ("x", "i"), ("q", "i"), ("s", "i"), ("a", "c"),
             ("b", "c"), ("k", "i"), ("w", "u"), ("d", "s")],
}
_PRESENT = {
    "nucdiv": "whpin", "sfs": "whpi", "ld": "whie", "diverge": "whpnti", "haplo": "whi", "snp": "whvizp",
    "tree": "whi",
}
_ATTR = {"f": "reffile", "h": "headfile", "m": "min_depth", "x": "max_depth", "q": "min_rmsQ",
         "s": "min_snpQ", "a": "min_mapQ", "b": "min_baseQ", "k": "min_sites", "w": "win_size",
         "o": "output", "n": "min_snps", "p": "outgroup", "d": "dist", "z": None}

_INT_RE = re.compile(r"^\s*[+-]?\d+")


def _is_int(s):
    return re.fullmatch(r"[+-]?\d+", s) is not None


def _is_float(s):
    try:
        float(s)
        return not s.strip().lower() in ("nan", "inf", "-inf", "+inf", "infinity")
    except ValueError:
        return False


def _convert(val, typ):
    """stringstream >> T; returns (value or None if nothing assigned, ok)."""
    if typ == "s":
        return val, True
    if typ == "c":
        return (ord(val[0]) if val else None), len(val) == 1
    if typ == "L":
        try:
            return float(val), True
        except ValueError:
            return None, False
    m = _INT_RE.match(val)
    if not m:
        return 0, False          # C++11 num_get writes 0 on a failed extraction
    v = int(m.group(0))
    if typ == "u" and v < 0:
        v &= 0xFFFFFFFF
    return v, m.end() == len(val)


def parse_args(cmd: str, argv: list[str]) -> Options:
    """argv excludes the subcommand name (it is GetOpt_pp's app name, skipped)."""
    if cmd not in _VALUE_OPTS:
        raise PopbamError(f"unrecognized command: {cmd}")
    o = Options(cmd=cmd)
    if cmd == "ld":
        o.min_sites = 10
    if cmd == "diverge":
        o.win_size = 1
    # tokenize (getopt_pp.cpp:66-140)
    toks = []      # [type, value]
    short = {}     # letter -> token index (last occurrence wins)
    any_opt = False
    for a in argv:
        if a.startswith("-") and len(a) > 1:
            if a[1] == "-":
                toks.append(["L" if len(a) > 2 else "G", a])
            elif _is_int(a):
                if len(a) > 2:
                    toks.append(["U" if any_opt else "G", a])
                else:
                    short[a[1]] = len(toks)
                    toks.append(["N", a])
            elif _is_float(a):
                toks.append(["U" if any_opt else "G", a])
            else:
                for ch in a[1:]:
                    short[ch] = len(toks)
                    toks.append(["S", ch])
            any_opt = True
        else:
            toks.append(["U" if any_opt else "G", a])
    for letter, typ in _VALUE_OPTS[cmd]:
        if letter not in short:
            continue
        i = short[letter] + 1
        if i >= len(toks) or toks[i][0] not in ("U", "A", "N"):
            continue  # NoArgs
        if toks[i][0] == "N":
            short.pop(toks[i][1][1], None)
        toks[i][0] = "A"
        val, ok = _convert(toks[i][1], typ)
        if not ok:
            o.errors.append(f"-{letter} {toks[i][1]}")
        attr = _ATTR[letter]
        if attr and val is not None:
            setattr(o, attr, val)
    present = set(short)
    if "w" in present and "w" in _PRESENT[cmd]:
        o.win_size = (o.win_size * 1000) & 0xFFFFFFFF
        o.flag |= BAM_WINDOW
    if "h" in present:
        o.flag |= BAM_HEADERIN
    if cmd in ("nucdiv", "sfs", "diverge", "snp") and "p" in present:
        o.flag |= BAM_OUTGROUP
    if "i" in present:
        o.flag |= BAM_ILLUMINA
    if cmd in ("nucdiv", "diverge") and "n" in present:
        o.flag |= BAM_MINPOPSAMPLE
    if cmd == "diverge" and "t" in present:
        o.flag |= BAM_SUBSTITUTE
    if cmd == "sfs" and "--theta" in argv:
        o.output |= 1   # extension: append S, theta_W and the spectrum (print_sfs never prints them)
    if cmd == "ld" and "e" in present:
        o.min_freq = 2
    if cmd == "snp" and "v" in present:
        o.flag |= BAM_VARIANT
    if cmd == "snp" and "z" in present:
        o.flag |= BAM_HETEROZYGOTE
    if cmd in ("diverge", "tree") and o.dist not in ("pdist", "jc"):
        raise PopbamError(f"{o.dist} is not a valid distance option")
    if cmd in ("ld", "haplo", "snp") and not 0 <= o.output <= 2:
        raise PopbamError("Not a valid output option")
    if cmd == "diverge" and not 0 <= o.output <= 1:
        raise PopbamError("Not a valid output option")
    glob = [v for t, v in toks if t in ("G", "U", "N")]
    if len(glob) < 2:
        raise PopbamError("Need to specify BAM file name")
    o.bamfile, o.region = glob[0], glob[1]
    return o


def parse_region(region: str, names: list[str], lengths: list[int]):
    """bam_parse_region (pop_utils.cpp:386-461) -> (tid, beg, end); raises on failure."""
    r = region.replace(" ", "").replace(",", "")
    l = len(r)
    name_end = r.find(":")
    if name_end < 0:
        name_end = l
    if name_end < l:
        coords = r[name_end + 1:]
        bad = any(ch not in "0123456789,-" for ch in coords) or coords.count("-") > 1
        if bad:
            name_end = l
        nm = r[:name_end]
        if nm not in names:
            if r not in names:
                raise PopbamError(f"Bad genome coordinates: {region}")
            nm = r
    else:
        nm = r
        if nm not in names:
            raise PopbamError(f"Bad genome coordinates: {region}")
    tid = names.index(nm)
    if name_end < l:
        coords = r[name_end + 1:]
        dash = coords.find("-")
        first = coords if dash < 0 else coords[:dash]
        last = coords if dash < 0 else coords[dash + 1:]
        beg = _atoi(first)
        if beg > 0:
            beg -= 1
        end = _atoi(last)
    else:
        beg, end = 0, lengths[tid]
    if beg > end:
        raise PopbamError(f"Bad genome coordinates: {region}")
    return tid, beg, end


def get_refid(text: str) -> str:
    """get_refid (pop_utils.cpp:463-498): the value of the header's first "AS:" tag, up to a
    tab or newline (the tree's name for the reference taxon)."""
    v = text.find("AS:")
    if v < 0:
        raise PopbamError("Unable to parse reference sequence name\n"
                          "Be sure the AS tag is defined in the sequence dictionary")
    u = v + 3
    w = u
    while w < len(text) and text[w] not in "\t\n":
        w += 1
    return text[u:w][:199]


def _atoi(s):
    m = _INT_RE.match(s)
    return int(m.group(0)) if m else 0


@dataclass
class SampleModel:
    samples: list
    pops: list
    rg2sample: dict
    sample_pop: list

    @property
    def n(self):
        return len(self.samples)

    def pop_masks(self):
        """assign_pops (popbam.cpp:145-171): (pop_mask[u64], pop_nsmpl)."""
        masks = [0] * len(self.pops)
        cnt = [0] * len(self.pops)
        for i, p in enumerate(self.sample_pop):
            masks[p] |= 1 << i
            cnt[p] += 1
        return masks, cnt


def parse_header(text: str, bamfile: str = "in.bam") -> SampleModel:
    """bam_smpl_add (pop_sample.cpp:15-107).  Searches for the next "\\tID:", "\\tSM:",
    "\\tPO:" anywhere after each "@RG", as the reference does."""
    samples, pops, rg2s, spop = [], [], {}, {}
    p = 0
    n = 0

    def field_at(i):
        j = i
        while j < len(text) and text[j] not in "\t\n":
            j += 1
        return text[i:j]

    while True:
        q = text.find("@RG", p)
        if q < 0:
            break
        p = q + 3
        qi = text.find("\tID:", p)
        ri = text.find("\tSM:", p)
        si = text.find("\tPO:", p)
        qi = qi + 4 if qi >= 0 else -1
        ri = ri + 4 if ri >= 0 else -1
        si = si + 4 if si >= 0 else -1
        if ri >= 0 and qi >= 0:
            rg, sm = field_at(qi), field_at(ri)
            if rg not in rg2s:
                if sm not in samples:
                    samples.append(sm)
                rg2s[rg] = samples.index(sm)
            if si >= 0:
                po = field_at(si)
                if sm not in spop:
                    if po not in pops:
                        pops.append(po)
                    spop[sm] = pops.index(po)
        else:
            break
        p = max(qi, ri, si)
        n += 1
    if n == 0:
        samples, pops, rg2s, spop = [bamfile], [bamfile], {}, {bamfile: 0}
    missing = [s for s in samples if s not in spop]
    if missing:
        raise PopbamError(f"Sample {missing[0]} not assigned to a population.\n"
                          "Please check BAM header file definitions")
    return SampleModel(samples, pops, rg2s, [spop[s] for s in samples])
