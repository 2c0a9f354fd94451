"""`popbam <cmd> [options] <in.bam> <region>` on the GPU: the drop-in command line.

Mirrors POPBAM's main (popbam.cpp:53-77) and main_<cmd> (e.g. pop_nucdiv.cpp:10-134) for the
subcommands snp, nucdiv, sfs, ld, diverge, haplo and tree:
  parseCommandLine (GetOpt_pp quirks, options.parse_args)
  -> checkBAM (popbam.cpp:95-143: BAM, optional -h header text, .bai, FASTA)
  -> bam_smpl_add (options.parse_header) -> bam_parse_region (options.parse_region)
  -> faidx_fetch_seq of the contig -> one pileup of the region (libpopbam_feed.so)
  -> pbg_run (libpopbam_gpu.so: consensus call, the reference's window loop, print_<cmd>).
stdout is the reference's TSV byte for byte; errors are reported like fatal_error
(pop_utils.cpp:510-519) with exit status 1.  `tree` (main_tree, pop_tree.cpp:10-136) takes its
per-window diff_matrix from the GPU and joins the (n+1)-taxon tree on the host.
"""
from __future__ import annotations

import os
import sys

from . import options as opt

COMMANDS = ("snp", "haplo", "diverge", "tree", "nucdiv", "ld", "sfs")

USAGE = """
Program: popbam (MI355X hot path: consensus call + window statistics on the GPU)

Usage:   popbam <command> [options] <in.bam> <region>

Command: snp         call SNPs
         haplo       haplotype-based statistics
         diverge     divergence from the reference
         tree        neighbour-joining tree per window (pdist or jc)
         nucdiv      nucleotide diversity (pi, dxy)
         ld          linkage disequilibrium (ZnS, omega_max, Wall's B/Q)
         sfs         site frequency spectrum (Tajima's D, Fay-Wu H)
"""


def _fatal(msg: str) -> int:
    sys.stderr.write("popbam runtime error:\n" + msg + "\nExiting program\n")
    return 1


def run(cmd: str, argv: list[str], device: int = 0) -> str:
    """One `popbam <cmd> argv...` invocation; returns stdout text (raises PopbamError)."""
    from . import engine, feed

    o = opt.parse_args(cmd, argv)
    if not os.path.exists(o.bamfile):
        raise opt.PopbamError(f"Cannot read BAM file {o.bamfile}")
    try:
        bam = feed.Bam(o.bamfile)
    except feed.FeedError as e:
        raise opt.PopbamError(f"Cannot read BAM file {o.bamfile}: {e}") from e
    try:
        header = bam.header_text
        if o.flag & opt.BAM_HEADERIN:
            with open(o.headfile, "rb") as f:
                header = f.read().decode("latin-1")
        if not bam.has_index:
            raise opt.PopbamError(f"Index file not available for BAM file {o.bamfile}")
        if not o.reffile or not os.path.exists(o.reffile):
            raise opt.PopbamError(f"Failed to load index for fastA reference file: {o.reffile}")
        sm = opt.parse_header(header, o.bamfile)
        refid = opt.get_refid(header) if cmd == "tree" else ""
        refs = bam.refs
        names, lengths = [r[0] for r in refs], [r[1] for r in refs]
        tid, beg, end = opt.parse_region(o.region, names, lengths)
        seq = feed.fasta_fetch(o.reffile, names[tid])
        if len(seq) < end:   # positions past the contig's sequence: no reference base
            seq = seq + b"N" * (end - len(seq))
        fallback = 0 if not sm.rg2sample else -1
        try:
            threads = int(os.environ.get("POPBAM_FEED_THREADS", min(8, os.cpu_count() or 1)))
            chunk = max(1 << 16, -(-(end - beg) // max(1, 4 * threads)))
            batch = bam.pileup(tid, beg, end, seq, sm.rg2sample, sm.n, o.max_depth, fallback,
                               threads=threads, chunk=chunk)
        except feed.FeedError as e:
            if e.code == feed.PBF_E_RG:
                raise opt.PopbamError("Problem assigning read group") from e
            raise opt.PopbamError(f"Failed to retrieve region {o.region}: {e}") from e
        return engine.run_command(o, sm, names[tid], beg, end, batch, pos0=beg, device=device, refid=refid)
    finally:
        bam.close()


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        sys.stderr.write(USAGE)
        return 1
    cmd = argv[0]
    if cmd not in COMMANDS:
        sys.stderr.write(f"Error: unrecognized command: {cmd}\n")
        return 1
    try:
        text = run(cmd, argv[1:], device=int(os.environ.get("POPBAM_DEVICE", "0")))
    except opt.PopbamError as e:
        return _fatal(str(e))
    sys.stdout.write(text)
    sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
