"""Host-side CLI mirror: GetOpt_pp quirks, bam_parse_region, @RG sample model."""
import pytest

from popbam_amd import options as opt


def test_defaults_nucdiv():
    o = opt.parse_args("nucdiv", ["-f", "ref.fa", "in.bam", "chr1"])
    assert (o.min_depth, o.max_depth, o.min_rmsQ, o.min_snpQ, o.min_mapQ, o.min_baseQ) == (3, 255, 25, 25, 13, 13)
    assert o.min_sites == 10 and o.flag == 0 and o.bamfile == "in.bam" and o.region == "chr1"


def test_window_kb_and_flag():
    o = opt.parse_args("sfs", ["-w", "10", "-f", "r.fa", "x.bam", "chr2:1-100"])
    assert o.win_size == 10000 and o.flag & opt.BAM_WINDOW


def test_unsigned_char_options_take_first_character():
    # getopt_pp.h:133-144 -- stringstream >> unsigned char
    assert opt.parse_args("nucdiv", ["-a", "7", "in.bam", "c"]).min_mapQ == ord("7")
    o = opt.parse_args("nucdiv", ["-b", "20", "in.bam", "c"])
    assert o.min_baseQ == ord("2") and o.errors


def test_flag_options_do_not_consume():
    o = opt.parse_args("ld", ["-w", "1", "-e", "in.bam", "chr1"])
    assert o.min_freq == 2 and o.bamfile == "in.bam" and o.region == "chr1"
    o = opt.parse_args("nucdiv", ["-i", "in.bam", "chr1"])
    assert o.flag & opt.BAM_ILLUMINA and o.bamfile == "in.bam"


def test_ld_n_is_min_snps_but_nucdiv_n_is_flag():
    assert opt.parse_args("ld", ["-n", "3", "in.bam", "c"]).min_snps == 3
    assert opt.parse_args("nucdiv", ["-n", "in.bam", "c"]).flag & opt.BAM_MINPOPSAMPLE


def test_missing_region_is_error():
    with pytest.raises(opt.PopbamError):
        opt.parse_args("nucdiv", ["-f", "r.fa", "in.bam"])


def test_bad_distance():
    with pytest.raises(opt.PopbamError):
        opt.parse_args("diverge", ["-d", "k2p", "in.bam", "c"])


@pytest.mark.parametrize("region,expect", [
    ("chr1", (0, 0, 1000)),
    ("chr1:101-200", (0, 100, 200)),
    ("chr1:1,001-2,000", (0, 1000, 2000)),
    ("chr1:500", (0, 499, 500)),          # single base (A.13)
    ("chr2:0-10", (1, 0, 10)),
])
def test_parse_region(region, expect):
    assert opt.parse_region(region, ["chr1", "chr2"], [1000, 50]) == expect


def test_parse_region_unknown():
    with pytest.raises(opt.PopbamError):
        opt.parse_region("chrX:1-5", ["chr1"], [10])


def test_header_sample_model():
    txt = ("@HD\tVN:1.0\n@RG\tID:a\tSM:s1\tPO:p2\n@RG\tID:b\tSM:s2\tPO:p1\n"
           "@RG\tID:c\tSM:s1\tPO:p2\n@RG\tID:d\tSM:s3\tPO:p2\n")
    sm = opt.parse_header(txt)
    assert sm.samples == ["s1", "s2", "s3"] and sm.pops == ["p2", "p1"]
    assert sm.rg2sample == {"a": 0, "b": 1, "c": 0, "d": 2}
    masks, cnt = sm.pop_masks()
    assert masks == [0b101, 0b010] and cnt == [2, 1]


def test_header_tags_searched_past_line_end():
    # pop_sample.cpp:37-42 strstr()s for the tags in the rest of the header text, so a
    # missing PO is taken from a later line and the parse resumes after it
    sm = opt.parse_header("@RG\tID:a\tSM:s1\n@RG\tID:b\tSM:s2\tPO:p\n")
    assert sm.samples == ["s1"] and sm.pops == ["p"]


def test_header_without_read_groups():
    sm = opt.parse_header("@HD\tVN:1.0\n", "x.bam")
    assert sm.samples == ["x.bam"] and sm.pops == ["x.bam"]


def test_get_refid():
    """get_refid (pop_utils.cpp:463-498): first AS: value up to a tab/newline, else fatal."""
    assert opt.get_refid("@HD\tVN:1.0\n@SQ\tSN:chr1\tLN:9\tAS:dm3\n") == "dm3"
    assert opt.get_refid("@SQ\tSN:chr1\tAS:ref one\tLN:9\n@SQ\tSN:chr2\tAS:other\n") == "ref one"
    with pytest.raises(opt.PopbamError, match="AS tag"):
        opt.get_refid("@SQ\tSN:chr1\tLN:9\n")


def test_tree_options():
    """treeData::parseCommandLine (pop_tree.cpp:590-631): -d pdist|jc, -k, -w in kb."""
    o = opt.parse_args("tree", ["-f", "r.fa", "-d", "jc", "-w", "5", "-k", "20", "in.bam", "chr1"])
    assert (o.dist, o.win_size, o.min_sites, o.flag & opt.BAM_WINDOW) == ("jc", 5000, 20, opt.BAM_WINDOW)
    assert opt.parse_args("tree", ["in.bam", "chr1"]).dist == "pdist"
    with pytest.raises(opt.PopbamError, match="not a valid distance option"):
        opt.parse_args("tree", ["-d", "k2p", "in.bam", "chr1"])
