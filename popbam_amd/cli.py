"""`popbam <cmd> [options] <in.bam> <region>` on the GPU: the drop-in command line.

Mirrors POPBAM's main (popbam.cpp:53-77) and main_<cmd> (e.g. pop_nucdiv.cpp:10-134) for the
subcommands snp, nucdiv, sfs, ld, diverge, haplo and tree:
  parseCommandLine (GetOpt_pp quirks, options.parse_args)
  -> checkBAM (popbam.cpp:95-143: BAM, optional -h header text, .bai, FASTA)
  -> bam_smpl_add (options.parse_header) -> bam_parse_region (options.parse_region)
  -> faidx_fetch_seq of the contig
  -> per block of whole windows: pieces of the pileup + per-sample partition + call_base's
     per-read loop (libpopbam_feed.so pbf_kstream_*, walked ahead by worker threads), each
     pushed to the GPU as it comes (libpopbam_gpu.so pbg_stream_*: copy + consensus call
     overlapping the walk), then the reference's window loop and print_<cmd>.
Multi-GPU: POPBAM_WORLD=N (or a torchrun launch) splits the window list into N contiguous
blocks, one rank process per GPU (popbam_amd.shard); rank 0 prints the blocks in order.
Blocks bound host and device memory by the block, not the region (the reference re-fetches
every window, pop_nucdiv.cpp:57-125); the text is the concatenation of the blocks' texts.
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


def window_blocks(beg: int, end: int, win_size: int, windowed: bool, block_sites: int):
    """Regions (beg', end') whose window loops print, in order, exactly the windows of
    (beg, end): blocks of whole windows covering about block_sites positions each
    (popbam_amd.shard's geometry).  Without -w the region is one window, one block."""
    from . import shard
    if not windowed:
        return [(beg, end)]
    nw = shard.num_windows(beg, end, win_size, True)
    per = max(1, block_sites // max(1, win_size))
    return [(beg + a * win_size, beg + min(nw, a + per) * win_size + 1) for a in range(0, nw, per)]


_CTX_CACHE: dict = {}
last_profile: dict = {}   # phase times of the last run() (bench.py's `cli` breakdown)


def _context(params, device: int):
    """One libpopbam_gpu context per (device, sample model + filters), kept across commands and
    blocks in this process: its tables (cal_coef, 33.5 MB) are built and uploaded once, and its
    stream slots, pinned staging and window plans serve every later run."""
    import ctypes as C
    from . import _lib
    key = (device, C.string_at(C.addressof(params), C.sizeof(params)))
    ctx = _CTX_CACHE.get(key)
    if ctx is None:
        if len(_CTX_CACHE) >= 4:   # a few sample models at most
            _CTX_CACHE.pop(next(iter(_CTX_CACHE))).close()
        if not _CTX_CACHE:
            import atexit
            atexit.register(_close_contexts)
        ctx = _CTX_CACHE[key] = _lib.Context(params, device, torch_first=False)
    return ctx


_FASTA_CACHE: dict = {}


def _reference(path: str, name: str) -> bytes:
    """The contig's reference sequence, kept across commands in this process like the context
    (keyed by the FASTA's path, size and modification time, so an edited file is read again)."""
    from . import feed
    st = os.stat(path)
    key = (os.path.realpath(path), st.st_size, st.st_mtime_ns, name)
    seq = _FASTA_CACHE.get(key)
    if seq is None:
        if len(_FASTA_CACHE) >= 4:
            _FASTA_CACHE.pop(next(iter(_FASTA_CACHE)))
        seq = _FASTA_CACHE[key] = feed.fasta_fetch(path, name)
    return seq


def _close_contexts():
    while _CTX_CACHE:
        _CTX_CACHE.popitem()[1].close()


def run(cmd: str, argv: list[str], device: int = 0, rank: int = 0, world: int = 1) -> str:
    """One `popbam <cmd> argv...` invocation; returns stdout text (raises PopbamError).
    With world > 1 this rank computes only its block of windows (popbam_amd.shard) and
    returns that block's text; the blocks concatenated in rank order are the full output.

    Per block of windows: the host feeder's workers walk the block's pieces ahead
    (pbf_kstream_*: BGZF inflate, pileup, per-sample partition, call_base's per-read loop) and
    each piece goes to the GPU as soon as it is handed out (pbg_stream_push: pinned staging,
    async copy into a device slot, the call), so the walk of piece i+1 overlaps the copy and
    call of piece i; pbg_stream_finish then runs the command's windows and prints them."""
    import time

    from . import _lib, engine, feed, shard

    t_start = time.perf_counter()
    prof = {"feeder": {}, "gpu": {}}
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
        if o.flag & opt.BAM_OUTGROUP and cmd in ("sfs", "diverge", "snp") and o.outgroup not in sm.samples:
            # checked right after bam_smpl_add (pop_sfs.cpp:37-50, pop_diverge.cpp:37-50, pop_snp.cpp:36-49)
            raise opt.PopbamError(f"Specified outgroup {o.outgroup} not found")
        refid = opt.get_refid(header) if cmd == "tree" else ""
        refs = bam.refs
        names, lengths = [r[0] for r in refs], [r[1] for r in refs]
        tid, beg, end = opt.parse_region(o.region, names, lengths)
        t0 = time.perf_counter()
        try:
            seq = _reference(o.reffile, names[tid])
        except feed.FeedError as e:
            raise opt.PopbamError(f"Failed to load index for fastA reference file: {o.reffile}: {e}") from e
        if len(seq) < end:   # positions past the contig's sequence: no reference base
            seq = seq + b"N" * (end - len(seq))
        prof["fasta_s"] = time.perf_counter() - t0
        fallback = 0 if not sm.rg2sample else -1
        windowed = bool(o.flag & opt.BAM_WINDOW)
        threads = int(os.environ.get("POPBAM_FEED_THREADS", min(16, os.cpu_count() or 1)))
        piece = int(os.environ.get("POPBAM_FEED_CHUNK", 1 << 16))
        nw_total = shard.num_windows(beg, end, o.win_size, windowed)
        rbeg, rend, ms0 = beg, end, nw_total
        if world > 1:
            reg = shard.shard_region(beg, end, o.win_size, windowed, rank, world)
            if reg is None:
                return ""
            (rbeg, rend), ms0 = reg, shard.ms_windows_for(beg, end, o.win_size, windowed, rank)
        block_sites = int(os.environ.get("POPBAM_BLOCK_SITES", 1 << 26))
        if cmd == "snp" and o.output == 0:   # consensus words: n * 8 bytes per position on device and host
            block_sites = min(block_sites, max(1 << 16, (1 << 30) // (8 * sm.n)))
        blocks = window_blocks(rbeg, rend, o.win_size, windowed, block_sites)
        if not blocks:   # no window: the reference's loop prints nothing
            return ""
        flt = engine.make_filter(o)
        t0 = time.perf_counter()
        ctx = _context(engine.make_params(o, sm), device)
        prof["context_s"] = time.perf_counter() - t0
        prof["feeder_threads"], prof["piece_sites"] = threads, piece
        parts = []
        t0 = time.perf_counter()
        for i, reg in enumerate(blocks):
            lo, hi = shard.positions_needed(reg[0], reg[1], o.win_size, windowed)
            hi = max(hi, lo)
            ms = (ms0 if i == 0 else -1) if len(blocks) > 1 or world > 1 else 0
            c = engine._Cmd(o, sm, names[tid], reg[0], reg[1], refid, ms)
            try:
                ks = bam.key_stream(tid, lo, hi, seq, sm.rg2sample, sm.n, engine.max_depth_of(o), flt, fallback,
                                    threads=threads, chunk=piece, win=o.win_size if windowed else 0)
            except feed.FeedError as e:
                raise opt.PopbamError(f"Failed to retrieve region {o.region}: {e}") from e
            with ks, _lib.Stream(ctx, [c.c], lo, hi - lo) as st:
                try:
                    while True:
                        p = ks.next()
                        if p is None:
                            break
                        try:
                            st.push(_lib.PbgPileup(p.n_sites, p.pos0, C_addr(p.ref), p.k, C_addr(p.rmsq),
                                                   C_addr(p.block_off), C_addr(p.keys)))
                        finally:
                            ks.release(p)
                except feed.FeedError as e:
                    if e.code == feed.PBF_E_RG:
                        raise opt.PopbamError("Problem assigning read group") from e
                    raise opt.PopbamError(f"Failed to retrieve region {o.region}: {e}") from e
                st.finish()
                parts.append(st.text(0))
                _accumulate(prof["feeder"], ks.profile())
                _accumulate(prof["gpu"], st.profile())
        prof["blocks_s"] = time.perf_counter() - t0
        prof["total_s"] = time.perf_counter() - t_start
        last_profile.clear()
        last_profile.update(prof)
        return "".join(parts)
    finally:
        bam.close()


def C_addr(ptr) -> int:
    """Address held by a ctypes pointer (0 for NULL)."""
    import ctypes as C
    return C.cast(ptr, C.c_void_p).value or 0


def _accumulate(acc: dict, d: dict):
    for k, v in d.items():
        acc[k] = acc.get(k, 0) + v


def _run_rank(cmd: str, argv: list[str]) -> int:
    """One rank of a sharded run (launched by _launch_ranks or torchrun): compute this rank's
    windows on GPU LOCAL_RANK, gather (status, text) to rank 0 over gloo, rank 0 prints.
    Every rank reaches the gather, also after an error, so a failing rank cannot hang the rest."""
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # the gloo runtime logs to file descriptor 1; keep stdout for the reference's TSV only
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        try:
            import torch
            ndev = max(1, torch.cuda.device_count())
            dev = int(os.environ.get("POPBAM_DEVICE", int(os.environ.get("LOCAL_RANK", rank)) % ndev))
            res = (0, run(cmd, argv, device=dev, rank=rank, world=world))
        except opt.PopbamError as e:
            res = (1, str(e))
        except Exception as e:   # any failure (GPU, feeder, ...) still reaches the gather
            res = (1, f"rank {rank}: {type(e).__name__}: {e}")
        parts = [None] * world if rank == 0 else None
        dist.gather_object(res, parts, dst=0)
    finally:
        dist.destroy_process_group()
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    if rank != 0:
        return res[0]
    for code, msg in parts:
        if code:
            return _fatal(msg)
    sys.stdout.write("".join(t for _, t in parts))
    sys.stdout.flush()
    return 0


def _launch_ranks(world: int, argv: list[str]) -> int:
    """POPBAM_WORLD=N: start N rank processes of this command (one per GPU, round-robin over the
    visible GPUs), rank 0's stdout is the command's stdout.  The launcher itself never touches
    the GPU; it starts children and returns the first non-zero status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), POPBAM_WORLD="1",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-m", "popbam_amd.cli", *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c), 0)


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        sys.stderr.write(USAGE)
        return 1
    cmd = argv[0]
    if cmd not in COMMANDS:
        sys.stderr.write(f"Error: unrecognized command: {cmd}\n")
        return 1
    # multi-GPU: POPBAM_WORLD=N starts N ranks; a torchrun launch (WORLD_SIZE > 1) is one rank
    world = int(os.environ.get("POPBAM_WORLD", "1"))
    if world > 1:
        return _launch_ranks(world, argv)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return _run_rank(cmd, argv[1:])
    try:
        text = run(cmd, argv[1:], device=int(os.environ.get("POPBAM_DEVICE", "0")))
    except opt.PopbamError as e:
        return _fatal(str(e))
    sys.stdout.write(text)
    sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
