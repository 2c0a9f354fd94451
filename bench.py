#!/usr/bin/env python3
"""Benchmark: Msites/s of the POPBAM hot path (per-site consensus call + nucdiv + sfs + ld
ZnS over 10 kb windows, 12 samples) on MI355X -- BASELINE.json configs[2]: synthetic 1 contig,
50 Msites x 12 samples.

One step = one pass of the hot path over one batch: the call kernel over every position of
the HBM-resident synthetic pileup (reads -> packed rows) followed by the window-statistics
kernel over all 4,999 windows.  Multi-GPU: one process per GPU (torchrun), each rank owns its
own 50 Msite shard (its own seed), no collective on the data path (weak scaling); only the
timing barrier and max-over-ranks reduction use torch.distributed.

Prints one JSON line (rank 0).  `roofline` is for the dominant kernel (call_scan_kernel, the
first kernel of the rows-only call): its algorithmic bytes per launch / its mean duration,
measured with HIP events the library records on the stream the kernel runs on
(pbg_set_kernel_timing / pbg_kernel_time).  `cpu_baseline` times the CPU oracle (C++ restatement of the reference
path, one core) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "Msites/sec (nucdiv+sfs+ld, 10kb win, 12 samples) at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
LAYOUT = "keys16"       # pileup batch layout the committed PMC profile was taken on


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sites", type=int, default=50_000_000, help="positions per GPU")
    ap.add_argument("--samples", type=int, default=12)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--window", type=int, default=10_000)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xC0FFEE02)
    ap.add_argument("--cpu-sample", type=int, default=60_000, help="positions for the CPU port baseline (0 = skip all)")
    ap.add_argument("--ref-sample", type=int, default=200_000, help="positions for the reference-binary baseline")
    ap.add_argument("--e2e-chunk", type=int, default=4_000_000,
                    help="config 2: positions per chunk of the measured host-input pass (0 = skip)")
    ap.add_argument("--e2e-passes", type=int, default=2)
    ap.add_argument("--cli-sample", type=int, default=200_000,
                    help="config 2: positions of the BAM the drop-in CLI is timed on (0 = skip)")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4),
                    help="BASELINE.json configs[i]: 2 = 50 Msites x 12 samples (the metric's config), "
                         "3 = whole genome 24 contigs x 125 Mbp x 24 samples, nucdiv+sfs+ld+diverge, "
                         "4 = deep panel 200 Msites x 96 samples, 1 kb windows every 500 bp, nucdiv+sfs+haplo EHHS")
    ap.add_argument("--step", type=int, default=500, help="config 4: window step (overlapping windows)")
    ap.add_argument("--contigs", type=int, default=24, help="config 3: contigs")
    ap.add_argument("--contig-len", type=int, default=125_000_000, help="config 3: positions per contig")
    ap.add_argument("--chunk", type=int, default=1 << 25, help="config 3: positions per streamed pileup chunk")
    ap.add_argument("--overlap", action="store_true",
                    help="configs[3]/[4]: generate chunk c+1 on a second stream beside the call of chunk c "
                         "(default: generate then call on one stream, so the call kernels run alone)")
    ap.add_argument("--pieces", type=int, default=1,
                    help="config 2: the contig's call in this many pieces (window borders), each piece's "
                         "statistics on a second stream beside the next piece's call (1 = call, then statistics)")
    args = ap.parse_args()
    if args.config == 3:
        if args.samples == 12:
            args.samples = 24
        if args.seed == 0xC0FFEE02:
            args.seed = 0xC0FFEE04
    if args.config == 4:
        if args.samples == 12:
            args.samples = 96
        if args.seed == 0xC0FFEE02:
            args.seed = 0xC0FFEE05
        if args.window == 10_000:
            args.window = 1000
        if args.contig_len == 125_000_000:
            args.contig_len = 200_000_000
        if args.chunk == 1 << 25:
            args.chunk = 1 << 23   # 96 samples: ~16 GB of keys per chunk buffer
        args.contigs = 1
    return args


def cpu_port(args):
    """Oracle (kind 'port', 1 core): three separate runs -- nucdiv, sfs, ld -- as the
    reference computes them, each re-calling every position, over the first --cpu-sample
    positions of the same synthetic pileup (no BAM decoding or pileup)."""
    import numpy as np

    import harness
    from popbam_amd import workload

    n, L = args.samples, args.cpu_sample
    batch = harness.synth_batch(args.seed, 0, L, n, args.depth)
    p = harness.oracle_params_from(workload.default_params(n))
    lib = harness.oracle()
    names = [f"s{i}".encode() for i in range(n)]
    pops = [b"popA", b"popB"]
    sn = (C.c_char_p * n)(*names)
    pn = (C.c_char_p * 2)(*pops)
    rd = np.ascontiguousarray(batch["reads"])
    tot = 0.0
    win = min(args.window, max(2, L // 4))
    if args.config == 4:   # overlapping windows: the oracle's call + its window statistics over the list
        step = args.step
        wins = [(a, a + win) for a in range(0, L - win + 1, step)]
        wb = np.array([a for a, _ in wins], np.int32)
        we = np.array([b for _, b in wins], np.int32)
        for cmd, out in ((4, 0), (6, 0), (1, 1)):   # nucdiv, sfs, haplo -o 1 (EHHS)
            c = harness.OrcCmd()
            c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq = cmd, out, 10, 10, 1
            c.chr_name = b"chr1"
            c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
            c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
            t0 = time.perf_counter()
            _, types, _, flags = harness.oracle_call(p, batch)
            buf = C.create_string_buffer(1 << 24)
            r = lib.orc_windows_from_sites(C.byref(p), C.byref(c), types.ctypes.data, flags.ctypes.data, len(wins),
                                           wb.ctypes.data, we.ctypes.data, buf, 1 << 24)
            tot += time.perf_counter() - t0
            assert r >= 0
        return {"value": round(L / tot / 1e6, 6), "unit": "Msites/s", "cores": 1, "kind": "port",
                "sample": f"first {L} positions of the same synthetic pileup ({n} samples, depth {args.depth}); "
                          f"oracle C++ restatement on 128-bit masks (the reference stops at 64 samples), nucdiv, sfs "
                          f"and haplo EHHS as 3 separate passes (each re-calls all sites), {win} bp windows every "
                          f"{step} bp; excludes BAM decode/pileup"}
    for cmd in (4, 6, 5):   # nucdiv, sfs, ld (popbam_func_t)
        c = harness.OrcCmd()
        c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq = cmd, 0, 10, 10, 1
        c.windowed, c.win_size, c.beg, c.end = 1, win, 0, L
        c.chr_name = b"chr1"
        c.sample_names = C.cast(sn, C.POINTER(C.c_char_p))
        c.pop_names = C.cast(pn, C.POINTER(C.c_char_p))
        buf = C.create_string_buffer(1 << 22)
        t0 = time.perf_counter()
        r = lib.orc_run(C.byref(p), C.byref(c), L, batch["ref"].ctypes.data, batch["depth"].ctypes.data,
                        rd.ctypes.data, buf, 1 << 22)
        tot += time.perf_counter() - t0
        assert r >= 0
    return {"value": round(L / tot / 1e6, 6), "unit": "Msites/s", "cores": 1, "kind": "port",
            "sample": f"first {L} positions of the same synthetic pileup ({n} samples, depth {args.depth}); "
                      f"oracle C++ restatement, nucdiv+sfs+ld as 3 separate passes (each re-calls all sites), "
                      f"{win} bp windows; excludes BAM decode/pileup"}


def cpu_baseline(args):
    """POPBAM itself (oracle/_ref/popbam, built from /root/reference) on a BAM of the same
    synthetic genome (tests/ref_baseline.py): nucdiv, sfs and ld as three processes, wall times
    summed, on the first --ref-sample positions; plus P region-sharded processes per command
    (P = the host's CPU share, at most 16).  The oracle port's rate is reported beside it."""
    import ref_baseline
    port = cpu_port(args)
    if args.config == 4 or not ref_baseline.available():   # the reference cannot hold 96 samples
        return port
    L, n = args.ref_sample, args.samples
    d = ref_baseline.make_inputs(f"/tmp/popbam_refbase_v3_{args.seed:x}_{L}_{n}", args.seed, L, n)
    procs = max(1, min(16, os.cpu_count() or 1))
    t = ref_baseline.time_reference(d, L, args.window, procs)
    out = {"value": round(L / t["single_total_s"] / 1e6, 6), "unit": "Msites/s", "cores": 1, "kind": "reference",
           "sample": f"oracle/_ref/popbam (POPBAM 0.3 built from /root/reference) nucdiv, sfs, ld -w "
                     f"{args.window // 1000} as 3 processes (wall {t['single_total_s']:.2f} s summed) on a BAM of "
                     f"positions [0, {L}) of the same synthetic genome: {n} samples, 100 bp reads every 10 bp "
                     f"(depth 10), baseQ 40, mapQ 60, 2 populations; includes BAM decode + pileup",
           "port": port}
    if "parallel_total_s" in t:
        out["all_cores"] = {"value": round(L / t["parallel_total_s"] / 1e6, 6), "cores": t["procs"],
                            "sample": f"{t['procs']} region-sharded processes per command, concurrent "
                                      f"(wall {t['parallel_total_s']:.2f} s summed over the 3 commands)"}
    return out


def pcie_rate(torch, batch_bytes: int, step_s: float, sites: int) -> dict:
    """The host-buffer boundary (pbg_run / the CLI hand the batch over in host memory): measured
    pinned host -> device bandwidth, and the rate the hot path would reach with the batch's
    bytes crossing PCIe, serially (copy, then call + stats) and double-buffered (copy of batch
    i+1 under the compute of batch i).  Never `value`: that is with the input resident."""
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        d.copy_(h, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    gbps = 4 * n / (e0.elapsed_time(e1) * 1e-3) / 1e9
    copy_s = batch_bytes / (gbps * 1e9)
    del h, d
    return {"h2d_GBps": round(gbps, 2), "batch_bytes": batch_bytes, "copy_ms": round(copy_s * 1e3, 2),
            "Msites_per_s_serial": round(sites / (copy_s + step_s) / 1e6, 2),
            "Msites_per_s_overlapped": round(sites / max(copy_s, step_s) / 1e6, 2)}


def end_to_end(args, torch, hp, stream) -> dict:
    """Measured host-input rate: the same contig handed over in
    pinned HOST memory, streamed host -> device in chunks of whole windows on a copy stream
    while the previous chunk is called and its windows computed (workload.HostStream, double
    buffered); wall time of whole passes.  The pass's rows and window outputs are checked
    against the HBM-resident step's."""
    want_rows = hp.rows.clone()
    want = {k: hp.out.t[k].clone() for k in ("num_sites", "segsites", "pi", "td", "ld_val")}
    host = hp.to_host()
    hs = hp.host_stream(host, args.e2e_chunk, args.window)
    hp.rows.zero_()
    for k in want:
        hp.out.t[k].zero_()
    hs.run(stream)   # warmup pass (plans, slots)
    torch.cuda.synchronize()
    same = bool(torch.equal(hp.rows, want_rows)) and all(bool(torch.equal(hp.out.t[k], v)) for k, v in want.items())
    passes = max(1, args.e2e_passes)
    t0 = time.perf_counter()
    for _ in range(passes):
        hs.run(stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / passes
    del host
    return {"Msites_per_s": round(args.sites / dt / 1e6, 2), "ms_per_pass": round(dt * 1e3, 2),
            "h2d_bytes_per_pass": hs.h2d_bytes, "h2d_GBps_effective": round(hs.h2d_bytes / dt / 1e9, 2),
            "chunk_sites": hs.chunk, "chunks": len(hs.chunks), "passes": passes,
            "matches_resident": same,
            "how": "pinned host batch (SURVEY 8(d) layout) -> H2D on a copy stream into two device slots, "
                   "pbg_call_sites + pbg_window_stats per chunk on the compute stream; wall time per pass"}


def cli_rate(args) -> dict:
    """The drop-in command line on a real BAM: `bin/popbam nucdiv|sfs|ld -f ref.fa -w 10 in.bam
    chr1` over the same BAM the reference baseline reads (tests/ref_baseline.py, the first
    --cli-sample positions), each as a fresh process (wall, including interpreter and GPU
    start-up) and in-process (popbam_amd.cli.run: BAM decode + pileup + key batch on the host
    feeder's threads, then the GPU), stdout compared with POPBAM's own."""
    import subprocess

    import ref_baseline
    from popbam_amd import cli
    L, n = args.cli_sample, args.samples
    d = ref_baseline.make_inputs(f"/tmp/popbam_refbase_v3_{args.seed:x}_{L}_{n}", args.seed, L, n)
    win_kb = str(args.window // 1000)
    threads = int(os.environ.get("POPBAM_FEED_THREADS", min(8, os.cpu_count() or 1)))
    res = {"sites": L, "samples": n, "feeder_threads": threads, "commands": {}}
    tot_proc = tot_in = 0.0
    same = True
    for c in ("nucdiv", "sfs", "ld"):
        argv = [c, "-f", "ref.fa", "-w", win_kb, "in.bam", "chr1"]
        t0 = time.perf_counter()
        p = subprocess.run([sys.executable, os.path.join(REPO, "bin", "popbam"), *argv], cwd=d, capture_output=True)
        t_proc = time.perf_counter() - t0
        cwd = os.getcwd()
        os.chdir(d)
        try:
            t0 = time.perf_counter()
            text = cli.run(c, argv[1:])
            t_in = time.perf_counter() - t0
        finally:
            os.chdir(cwd)
        ok = p.returncode == 0 and p.stdout.decode() == text
        if ref_baseline.available():
            r = subprocess.run([ref_baseline.REF_BIN, *argv], cwd=d, capture_output=True)
            ok = ok and r.stdout.decode() == text
        same &= ok
        res["commands"][c] = {"process_s": round(t_proc, 3), "in_process_s": round(t_in, 3)}
        tot_proc += t_proc
        tot_in += t_in
    res.update({"Msites_per_s_process": round(L / tot_proc / 1e6, 4), "Msites_per_s_in_process": round(L / tot_in / 1e6, 4),
                "identical_to_reference": same,
                "note": "3 commands summed, as the CPU baseline; a fresh process pays Python + torch import and "
                        "context creation; in-process is the feeder + GPU path alone"})
    return res


def max_over_ranks(dist, x: float) -> float:
    """The slowest rank's time (gloo, on the host)."""
    if not dist:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_genome(args, torch, dist, world, rank):
    """configs[3]: the whole synthetic genome (contigs x contig-len, 24 samples) streamed through
    HBM in double-buffered pileup chunks (popbam_amd.genome), contig-first shards across ranks,
    nucdiv + sfs + ld (ZnS) + diverge over 10 kb windows.  Strong scaling: the genome is fixed."""
    from popbam_amd import _lib, genome, workload
    SITE_BLOCK = _lib.PBG_SITE_BLOCK

    n = args.samples
    ctx = _lib.Context(workload.default_params(n), torch.cuda.current_device())
    lengths = [args.contig_len] * args.contigs
    segs, stats = genome.rank_plan(args.config, lengths, world, rank, args.window, args.step)
    gp = genome.GenomePass(ctx, segs, args.seed, args.depth, args.window, stats, args.chunk, serial=not args.overlap)
    for _ in range(args.warmup):
        gp.run()
    gp.synchronize()
    gp.key_total.zero_()
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 1), "pbg_set_kernel_timing")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gp.run()
    gp.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    kt, kn = C.c_double(0.0), C.c_uint32(0)
    ctx.check(ctx.lib.pbg_kernel_time(ctx.h, C.byref(kt), C.byref(kn)), "pbg_kernel_time")
    ct, cn = C.c_double(0.0), C.c_uint32(0)
    ctx.check(ctx.lib.pbg_call_time(ctx.h, C.byref(ct), C.byref(cn)), "pbg_call_time")
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 0), "pbg_set_kernel_timing")
    my_sites = gp.n_sites
    total_sites = sum(lengths)
    sb = gp.survey_bytes(args.steps)
    scan_ms = kt.value / max(1, kn.value)             # per chunk launch, beside the generator
    chunks = len(gp.chunks)
    achieved_pass = sb / chunks / (scan_ms * 1e-3) / 1e9 if chunks else 0.0
    call_ms_pass = ct.value / max(1, args.steps)
    # the same kernel on one resident chunk with nothing else on the GPU (untimed for `value`):
    # in the pass the generator's kernels share the CUs, which roughly halves the scan's rate
    gp._generate(0, 0)
    gp.synchronize()
    L0 = gp.chunks[0][2]
    nb0 = (L0 + SITE_BLOCK - 1) // SITE_BLOCK
    keys0 = int(gp.buf[0]["block_off"][nb0].item())
    sb0 = 2 * keys0 + 5 * L0 * n + L0 * (1 + ctx.row_bytes)
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 1), "pbg_set_kernel_timing")
    for _ in range(5):
        gp._call(0, 0)
    gp.synchronize()
    k1, n1 = C.c_double(0.0), C.c_uint32(0)
    ctx.check(ctx.lib.pbg_kernel_time(ctx.h, C.byref(k1), C.byref(n1)), "pbg_kernel_time")
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 0), "pbg_set_kernel_timing")
    scan_ms_alone = k1.value / max(1, n1.value)
    achieved_alone = sb0 / (scan_ms_alone * 1e-3) / 1e9
    out = None
    if rank == 0:
        value = total_sites * args.steps / elapsed / 1e6
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msites/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (counter-based pileup generated on device chunk by chunk, inside the timed region)",
            "config": {"workload": (f"configs[3]: synthetic whole genome {args.contigs} contigs x "
                                    f"{args.contig_len / 1e6:g} Mbp x {n} samples, consensus call + nucdiv + sfs + "
                                    f"ld(ZnS) + diverge, {args.window / 1e3:g} kb windows, sharded by contig")
                       if args.config == 3 else
                       (f"configs[4]: synthetic deep panel {args.contig_len / 1e6:g} Msites x {n} samples, consensus "
                        f"call + nucdiv + sfs + haplo EHHS, {args.window / 1e3:g} kb windows every {args.step} bp "
                        f"(overlapping), window blocks per rank with a {args.window - args.step} bp halo"),
                       "genome_sites": total_sites, "sites_rank0": my_sites, "samples": n, "mean_depth": args.depth,
                       "window": args.window, "windows_rank0": gp.n_windows, "chunk_sites": args.chunk,
                       "chunks_rank0": chunks, "parallelism": f"dp{world} (contig-first shards, no collective)"},
            "roofline": {"bound": "hbm", "kernel": "call_scan_kernel", "achieved": round(achieved_pass, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_pass / HBM_PEAK_GBS, 4),
                         "traffic": None, "bytes_per_launch": sb // max(1, chunks), "ms_per_launch": round(scan_ms, 4),
                         "bytes_basis": "SURVEY 8(d): sum over (position, sample) of 2k+5, +1 +row_bytes per position",
                         "measured_on": (f"every chunk launch of the timed pass ({chunks} per pass; library HIP "
                                         "events on the call stream)") +
                                        (", the next chunk's generator running beside it" if args.overlap else
                                         ", each chunk generated before its call on the same stream"),
                         "alone": {"ms_per_launch": round(scan_ms_alone, 4), "achieved": round(achieved_alone, 2),
                                   "frac": round(achieved_alone / HBM_PEAK_GBS, 4), "bytes_per_launch": sb0,
                                   "note": "chunk 0 resident in HBM, 5 launches with nothing else on the GPU"}},
            "call_stage": {"ms_per_pass": round(call_ms_pass, 3), "bytes_per_pass": sb,
                           "GBps": round(sb / (call_ms_pass * 1e-3) / 1e9, 2) if call_ms_pass else None,
                           "Msites_per_s_call_only": round(my_sites / (call_ms_pass * 1e-3) / 1e6, 2) if call_ms_pass else None},
            "note": "value includes the on-device generation of every pileup chunk (the input does not fit "
                    "HBM: ~1.8 TB of keys); call_stage is the call kernels alone (library HIP events)",
            "pass_mode": "overlapped (two streams)" if args.overlap else "serial (generate, then call, per chunk)",
        }
        out["cpu_baseline"] = cpu_baseline(args) if (world == 1 and args.cpu_sample > 0) else None
        if out["cpu_baseline"]:
            out["x_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    ctx.close()


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # gloo (host) for the timing barrier and the max over ranks: the data path has no
        # collective, so RCCL is never initialised
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)

    if args.config in (3, 4):
        bench_genome(args, torch, dist, world, rank)
        if dist:
            dist.destroy_process_group()
        return

    from popbam_amd import _lib, workload

    n = args.samples
    params = workload.default_params(n)
    ctx = _lib.Context(params, torch.cuda.current_device())
    # each rank: its own 50 Msite contig of the synthetic genome (weak scaling)
    syn = workload.SynthPileup(ctx, args.sites, args.depth, args.seed, contig=rank)
    wins = workload.reference_windows(0, args.sites, args.window)
    stats = _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS
    hp = workload.HotPath(ctx, syn, wins, stats)
    stream = torch.cuda.current_stream()
    stats_stream = torch.cuda.Stream()
    pts = hp.pipeline(args.pieces) if args.pieces > 1 else [0, args.sites]

    def step():
        if args.pieces > 1:
            hp.step_pipelined(stream, stats_stream)
        else:
            hp.step(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # HIP events around the dominant kernel (call_scan_kernel), recorded by the library on the
    # stream it launches on (torch's events only bracket whole stages)
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 1), "pbg_set_kernel_timing")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    kt, kn = C.c_double(0.0), C.c_uint32(0)
    ctx.check(ctx.lib.pbg_kernel_time(ctx.h, C.byref(kt), C.byref(kn)), "pbg_kernel_time")
    ct, cn = C.c_double(0.0), C.c_uint32(0)
    ctx.check(ctx.lib.pbg_call_time(ctx.h, C.byref(ct), C.byref(cn)), "pbg_call_time")
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 0), "pbg_set_kernel_timing")

    # stage breakdown (untimed for `value`): the call of every piece, then the statistics of
    # every piece, serially on one stream (the same launches as the timed steps)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(3)]
    for e0, e1, e2 in ev:
        e0.record(stream)
        hp.call_pieces(stream) if args.pieces > 1 else hp.call(stream)
        e1.record(stream)
        hp.stats_pieces(stream) if args.pieces > 1 else hp.window_stats(stream)
        e2.record(stream)
    torch.cuda.synchronize()
    call_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    stats_ms = sum(b.elapsed_time(c) for _, b, c in ev) / len(ev)
    scan_ms = kt.value / max(1, kn.value)            # per call_scan_kernel launch (one per piece)
    total_sites = args.sites * world * args.steps
    value = total_sites / elapsed / 1e6
    call_lib_ms = ct.value / max(1, args.steps)      # whole call stage per step (all pieces)
    call_bytes = syn.survey_bytes()          # sum(2k + 5) + 1 + row_bytes per position
    scan_bytes = call_bytes
    layout_bytes = syn.layout_bytes_scan()
    scan_bytes_launch = scan_bytes * args.steps // max(1, kn.value)   # per launch (the pieces' mean)
    achieved = scan_bytes * args.steps / (kt.value * 1e-3) / 1e9
    stats_bytes = args.sites * ctx.row_bytes

    # per-launch HBM traffic from rocprofv3 PMC counters, when a profile of this code is committed
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_call_scan_kernel.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                d = json.load(f)
            if (d.get("sites") == args.sites and d.get("samples") == n and d.get("depth") == args.depth
                    and d.get("layout") == LAYOUT and d.get("pieces", 1) == len(pts) - 1):
                traffic = d.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msites/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (counter-based pileup resident in HBM, generated on device)",
            "config": {"workload": (("configs[2]: " if (args.sites, n, args.window) == (50_000_000, 12, 10_000)
                                     else "off-metric shape: ") +
                                    f"synthetic 1 contig x {args.sites / 1e6:g} Msites x {n} samples per GPU, "
                                    f"consensus call + nucdiv + sfs + ld(ZnS), {args.window / 1e3:g} kb windows"),
                       "sites_per_gpu": args.sites, "samples": n, "mean_depth": args.depth,
                       "window": args.window, "windows_per_gpu": len(wins), "keys_per_gpu": syn.n_keys,
                       "parallelism": f"dp{world} (independent window-range shards, no collective)",
                       "pieces": len(pts) - 1},
            "roofline": {"bound": "hbm", "kernel": "call_scan_kernel", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "bytes_per_launch": scan_bytes_launch, "ms_per_launch": round(scan_ms, 4),
                         "bytes_basis": "SURVEY 8(d): sum over (position, sample) of 2k+5, +1 +row_bytes per position",
                         "layout_bytes_per_launch": layout_bytes,
                         "frac_layout": round(layout_bytes * args.steps / (kt.value * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "call_stage": {"ms_serial": round(call_ms, 4), "ms_library_events": round(call_lib_ms, 4),
                           "bytes": call_bytes, "GBps": round(call_bytes / (call_lib_ms * 1e-3) / 1e9, 2),
                           "frac": round(call_bytes / (call_lib_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "kernels": "call_scan + call_slow + call_deepq + call_overflow + call_fold"},
            "window_stats": {"ms_serial": round(stats_ms, 4), "rows_bytes": stats_bytes,
                             "GBps": round(stats_bytes / (stats_ms * 1e-3) / 1e9, 2),
                             "Msites_per_s_stats_only": round(args.sites / (stats_ms * 1e-3) / 1e6, 2)},
        }
        if world == 1:
            out["pcie_inclusive"] = pcie_rate(torch, layout_bytes - args.sites * n, elapsed / args.steps, args.sites)
            if args.e2e_chunk > 0 and args.cpu_sample > 0:   # --cpu-sample 0 (profiling runs) skips the extras
                out["end_to_end"] = end_to_end(args, torch, hp, stream)
            if args.cli_sample > 0 and args.cpu_sample > 0:
                out["cli"] = cli_rate(args)
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(args)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 0), "pbg_set_kernel_timing")
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
