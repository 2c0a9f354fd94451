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
CALL_KERNELS = ("call_scan_kernel", "call_slow_kernel", "call_deepq_kernel", "call_overflow_kernel",
                "call_pend_fold_kernel")


def source_hash() -> str:
    """sha256 over the sources libpopbam_gpu.so is built from (popbam_amd/csrc minus the host
    feeder, which is its own library; the headers; include/popbam_gpu.h): a PMC profile counts
    for this build only if it records the same hash."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(REPO, "popbam_amd", "csrc")
    files = sorted([f for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp"))
                    if os.path.basename(f) != "feeder.cpp"] +
                   glob.glob(os.path.join(csrc, "*.h")) + [os.path.join(csrc, "Makefile"),
                                                          os.path.join(REPO, "include", "popbam_gpu.h")])
    for f in files:
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(config: int, shape: dict) -> dict | None:
    """Per-launch HBM bytes of the call kernels from rocprofv3 counters (FETCH_SIZE x 2 +
    WRITE_SIZE, separate --pmc passes; tools/pmc_traffic.py), accepted only when the profile
    was taken on this source tree (same source_hash) and this shape; else None."""
    path = os.path.join(REPO, "profiles", f"pmc_traffic_c{config}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None
    if d.get("src_sha") != source_hash():
        return None
    if any(d.get("shape", {}).get(k) != v for k, v in shape.items()):
        return None
    d["file"] = os.path.relpath(path, REPO)
    return d


HBM_ACHIEVABLE_GBS = 6290.0   # measured float4-copy rate (MI355X_MICROARCH.md), the most HBM delivers


def traffic_split(traffic: int | None, ms: float) -> dict | None:
    """What a counted `traffic` (FETCH_SIZE x 2 + WRITE_SIZE, bytes per launch) can mean at the
    launch's duration.  FETCH_SIZE counts the L2's fabric requests, Infinity-Cache (MALL) hits
    included (MI355X_MICROARCH.md, HBM / rocprofv3 section), so the count is an upper bound of the
    HBM bytes: at most HBM_ACHIEVABLE_GBS x duration of it can have come from HBM, the rest was served
    by the Infinity Cache.  A ratio above 1 over the algorithmic bytes is then not all HBM waste."""
    if not traffic or ms <= 0:
        return None
    cap = HBM_ACHIEVABLE_GBS * 1e9 * ms * 1e-3
    return {"counted_GBps": round(traffic / (ms * 1e-3) / 1e9, 1), "hbm_achievable_GBps": HBM_ACHIEVABLE_GBS,
            "hbm_bytes_at_most": int(min(traffic, cap)), "infinity_cache_bytes_at_least": int(max(0.0, traffic - cap)),
            "note": "traffic = L2 fabric requests (FETCH_SIZE x 2 + WRITE_SIZE), Infinity-Cache hits included; "
                    "at this launch's duration HBM can deliver at most hbm_bytes_at_most of it (6.29 TB/s "
                    "achievable), the rest came from the 256 MiB Infinity Cache"}


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
    ap.add_argument("--e2e-chunk", type=int, default=0,
                    help="config 2: positions per device slot of the measured host-input run (0 = the library's "
                         "default, -1 = skip)")
    ap.add_argument("--e2e-passes", type=int, default=2)
    ap.add_argument("--cli-sample", type=int, default=5_000_000,
                    help="config 2: positions of the BAM the drop-in CLI is timed on (0 = skip)")
    ap.add_argument("--parity-windows", type=int, default=20,
                    help="after timing: windows of the run checked against the CPU oracle (0 = skip)")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4),
                    help="BASELINE.json configs[i]: 2 = 50 Msites x 12 samples (the metric's config), "
                         "3 = whole genome 24 contigs x 125 Mbp x 24 samples, nucdiv+sfs+ld+diverge, "
                         "4 = deep panel 200 Msites x 96 samples, 1 kb windows every 500 bp, nucdiv+sfs+haplo EHHS")
    ap.add_argument("--step", type=int, default=500, help="config 4: window step (overlapping windows)")
    ap.add_argument("--contigs", type=int, default=24, help="config 3: contigs")
    ap.add_argument("--contig-len", type=int, default=125_000_000, help="config 3: positions per contig")
    ap.add_argument("--chunk", type=int, default=None, help="configs[3]/[4]: positions per streamed pileup chunk (default 2^27 serial or 2^25 --overlap / 2^23)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: each rank builds its shard plan, joins the gloo barrier / max-over-ranks timing "
                         "and rank 0 prints the line with value null (tests the --gpus N launch on CPU)")
    ap.add_argument("--allow-variant", action="store_true",
                    help="accept a library whose pbg_build_info() is not 'product' (bounds / experiment builds); "
                         "the line then says so in build.kind and is not a product measurement")
    ap.add_argument("--overlap", action="store_true",
                    help="configs[3]/[4]: generate chunk c+1 on a second stream beside the call of chunk c "
                         "(default: generate then call on one stream, so the call kernels run alone)")
    ap.add_argument("--pieces", type=int, default=1,
                    help="config 2: the contig's call in this many pieces (window borders), each piece's "
                         "statistics on a second stream beside the next piece's call (1 = call, then statistics)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.chunk is None:
        # one chunk per 125 Mbp contig (~64 GB of keys in the one serial buffer) for configs[3]'s
        # serial pass, 2^25 when two buffers alternate (--overlap), 2^23 at configs[4]'s 96 samples
        args.chunk = {3: (1 << 25) if args.overlap else (1 << 27), 4: 1 << 23}.get(args.config, 1 << 25)
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


def host_cpu_share() -> dict:
    """The host cores this run may use: the machine's count (os.cpu_count / nproc), the scheduler
    affinity of this process, the cgroup CPU quota, and OMP_NUM_THREADS (the GPU pool's per-box
    share).  `cores` = the smallest of them: the count every all-core figure below runs with."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    lim = [("affinity", aff)] + ([("cgroup_quota", quota)] if quota else []) + ([("OMP_NUM_THREADS", omp)] if omp else [])
    by, cores = min(lim, key=lambda x: x[1])
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "omp_num_threads": omp, "cores": cores,
            "bounded_by": by}


_ALL_CORES: dict = {}   # POPBAM region-sharded on every usable core, per (BAM dir): measured once


def popbam_all_cores(d: str, L: int, win: int) -> dict:
    """POPBAM itself (oracle/_ref/popbam) as P concurrent region-sharded processes per command
    (P = host_cpu_share()['cores'] shards of whole windows), nucdiv + sfs + ld summed; stdout of
    the shards concatenated = the command's text (the CLI leg compares it with ours)."""
    import ref_baseline
    if d not in _ALL_CORES:
        share = host_cpu_share()
        t = ref_baseline.time_reference(d, L, win, share["cores"], single=False, capture=True)
        _ALL_CORES[d] = {"Msites_per_s": round(L / t["parallel_total_s"] / 1e6, 4), "cores": share["cores"],
                         "processes": t["procs"], "wall_s": round(t["parallel_total_s"], 2),
                         "per_command_s": {c: round(v, 3) for c, v in t["parallel"].items()},
                         "host": share, "texts": t["texts"]}
    return _ALL_CORES[d]


def cpu_baseline(args):
    """POPBAM itself (oracle/_ref/popbam, built from /root/reference) on a BAM of the same
    synthetic genome (tests/ref_baseline.py): nucdiv, sfs and ld as three processes, wall times
    summed, on the first --ref-sample positions (one core); and on every usable host core
    (host_cpu_share) as region-sharded processes per command over the --cli-sample BAM, which has
    enough windows for one shard per core.  The oracle port's rate is reported beside it."""
    import ref_baseline
    port = cpu_port(args)
    if args.config == 4 or not ref_baseline.available():   # the reference cannot hold 96 samples
        return port
    L, n = args.ref_sample, args.samples
    d = ref_baseline.make_inputs(f"/tmp/popbam_refbase_v5_{args.seed:x}_{L}_{n}", args.seed, L, n)
    t = ref_baseline.time_reference(d, L, args.window, 1)
    out = {"value": round(L / t["single_total_s"] / 1e6, 6), "unit": "Msites/s", "cores": 1, "kind": "reference",
           "sample": f"oracle/_ref/popbam (POPBAM 0.3 built from /root/reference) nucdiv, sfs, ld -w "
                     f"{args.window // 1000} as 3 processes (wall {t['single_total_s']:.2f} s summed) on a BAM of "
                     f"positions [0, {L}) of the same synthetic genome: {n} samples, 100 bp reads every 10 bp "
                     f"(depth 10), baseQ 40, mapQ 60, 2 populations; includes BAM decode + pileup",
           "host": host_cpu_share(), "port": port}
    LA = max(args.cli_sample, L)
    da = ref_baseline.make_inputs(f"/tmp/popbam_refbase_v5_{args.seed:x}_{LA}_{n}", args.seed, LA, n)
    ac = popbam_all_cores(da, LA, args.window)
    out["all_cores"] = {"value": ac["Msites_per_s"], "cores": ac["cores"], "processes": ac["processes"],
                        "sample": f"{ac['processes']} region-sharded processes per command on {ac['cores']} usable "
                                  f"cores ({ac['host']['bounded_by']}), concurrent, over positions [0, {LA}) "
                                  f"(wall {ac['wall_s']:.2f} s summed over the 3 commands)"}
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


def stat_cmds(args, n: int, n_pops: int, lo: int, hi: int):
    """PbgCmd structures for `popbam nucdiv|sfs|ld -w <window>` over [lo, hi) (the metric's three
    commands) and the names they point at (kept alive by the caller)."""
    from popbam_amd import _lib
    keep = [b"chr1", (C.c_char_p * n)(*[f"s{i}".encode() for i in range(n)]),
            (C.c_char_p * n_pops)(*[f"p{i}".encode() for i in range(n_pops)])]
    cmds = []
    for cmd_id in (4, 6, 5):   # nucdiv, sfs, ld (popbam_func_t)
        c = _lib.PbgCmd()
        c.cmd, c.output, c.min_sites, c.min_snps, c.min_freq = cmd_id, 0, 10, 10, 1
        c.windowed, c.win_size, c.beg, c.end = 1, args.window, lo, hi
        c.chr_name = keep[0]
        c.sample_names = C.cast(keep[1], C.POINTER(C.c_char_p))
        c.pop_names = C.cast(keep[2], C.POINTER(C.c_char_p))
        c.refid = b"ref"
        cmds.append(c)
    return cmds, keep


def resident_texts(ctx, hp, cmds, wins) -> list:
    """print_<stat> of the HBM-resident step's window outputs (pbg_format) for each command."""
    import numpy as np
    from popbam_amd import _lib
    host = {k: v.cpu().numpy() for k, v in hp.out.t.items()}
    o = _lib.PbgWindowOut()
    for k, _ in _lib.PbgWindowOut._fields_:
        setattr(o, k, host[k].ctypes.data)
    wb = np.array([a for a, _ in wins], np.int32)
    we = np.array([b for _, b in wins], np.int32)
    out = []
    for c in cmds:
        need = C.c_size_t(0)
        ctx.lib.pbg_format(ctx.h, C.byref(c), C.byref(o), len(wins), wb.ctypes.data, we.ctypes.data, None, 0, C.byref(need))
        buf = C.create_string_buffer(need.value)
        ctx.check(ctx.lib.pbg_format(ctx.h, C.byref(c), C.byref(o), len(wins), wb.ctypes.data, we.ctypes.data, buf,
                                     need.value, C.byref(need)), "pbg_format")
        out.append(buf.value.decode())
    return out


def end_to_end(args, torch, ctx, hp, wins) -> dict:
    """Measured host-input rate through the C-ABI: the contig's key
    batch handed over in pinned HOST memory to a streamed run (pbg_stream_open / _push /
    _finish: chunks copied host -> device on a copy stream into two device slots while the
    previous chunk is called, then nucdiv + sfs + ld over every window and their TSV), wall time
    of whole runs, open to text.  The run's rows and texts are checked against the HBM-resident
    step's (rows bit for bit, texts byte for byte)."""
    from popbam_amd import _lib
    n, np_ = ctx.params.n_samples, ctx.params.n_pops
    cmds, keep = stat_cmds(args, n, np_, 0, args.sites)
    want = resident_texts(ctx, hp, cmds, wins)
    host = hp.to_host()
    piece = _lib.PbgPileup(args.sites, 0, host["ref"].data_ptr(), host["k"].data_ptr(), host["rmsq"].data_ptr(),
                           host["block_off"].data_ptr(), host["keys"].data_ptr())

    def run():
        with _lib.Stream(ctx, cmds, 0, args.sites, args.e2e_chunk) as st:
            st.push(piece)
            st.finish()
            return st, [st.text(i) for i in range(len(cmds))], st.profile()

    rows = torch.empty_like(hp.rows)
    with _lib.Stream(ctx, cmds, 0, args.sites, args.e2e_chunk) as st:   # warmup: slots, plans
        st.push(piece)
        st.finish()
        st.rows_into(rows.data_ptr(), rows.numel())
        texts = [st.text(i) for i in range(len(cmds))]
    torch.cuda.synchronize()
    same = bool(torch.equal(rows, hp.rows)) and texts == want
    passes = max(1, args.e2e_passes)
    t0 = time.perf_counter()
    for _ in range(passes):
        _, texts, prof = run()
    dt = (time.perf_counter() - t0) / passes
    same = same and texts == want
    compact = end_to_end_compact(args, torch, ctx, hp, cmds, want, host)
    del host
    return {"Msites_per_s": round(args.sites / dt / 1e6, 2), "ms_per_run": round(dt * 1e3, 2),
            "Msites_per_s_compact": compact["Msites_per_s"], "compact": compact,
            "h2d_bytes_per_run": prof["h2d_bytes"], "h2d_GBps_effective": round(prof["h2d_bytes"] / dt / 1e9, 2),
            "chunks": prof["chunks"], "pinned_chunks": prof["pinned_chunks"],
            "ms_h2d_device": round(prof["ms_h2d"], 2), "ms_call_device": round(prof["ms_call"], 2),
            "ms_finish": round(prof["ms_finish"], 2), "runs": passes, "matches_resident": same,
            "how": "C-ABI pbg_stream_*: pinned host key batch (SURVEY 8(d) layout) -> H2D chunks on a copy stream "
                   "into two device slots, pbg_call_sites per chunk on the compute stream, then nucdiv + sfs + ld "
                   "over all windows and their TSV; wall time per run (open -> three texts)"}


def end_to_end_compact(args, torch, ctx, hp, cmds, want, host) -> dict:
    """The same streamed run with COMPACT pieces (pbg_stream_push_compact): the reference-only
    tasks' keys stay on the host (rmsq bit 31 flags them; the feeder flags them as it packs, here
    pbf_compact converts the pinned host batch once, before timing), so far fewer bytes cross
    PCIe.  Rows and texts must equal the resident step's."""
    import numpy as np
    from popbam_amd import _lib, feed
    n = ctx.params.n_samples
    full = {k: host[k].numpy() for k in ("ref", "k", "rmsq", "keys", "block_off")}
    full["k"] = full["k"].reshape(args.sites, n)
    full["rmsq"] = full["rmsq"].reshape(args.sites, n)
    t0 = time.perf_counter()
    c = feed.compact(full, n, ctx.k_bytes)
    t_conv = time.perf_counter() - t0
    signed = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32, np.dtype(np.uint64): np.int64}
    pin = {}
    for k, v in c.items():
        if k == "pos0":
            continue
        a = np.ascontiguousarray(v).reshape(-1)
        pin[k] = torch.from_numpy(a.view(signed.get(a.dtype, a.dtype))).pin_memory()
    del c, full
    piece = _lib.PbgPileup(args.sites, 0, pin["ref"].data_ptr(), pin["k"].data_ptr(), pin["rmsq"].data_ptr(),
                           pin["block_off"].data_ptr(), pin["keys"].data_ptr())

    def run():
        with _lib.Stream(ctx, cmds, 0, args.sites, args.e2e_chunk) as st:
            st.push(piece, compact=True)
            st.finish()
            return st, [st.text(i) for i in range(len(cmds))], st.profile()

    rows = torch.empty_like(hp.rows)
    with _lib.Stream(ctx, cmds, 0, args.sites, args.e2e_chunk) as st:   # warmup
        st.push(piece, compact=True)
        st.finish()
        st.rows_into(rows.data_ptr(), rows.numel())
        texts = [st.text(i) for i in range(len(cmds))]
    torch.cuda.synchronize()
    same = bool(torch.equal(rows, hp.rows)) and texts == want
    passes = max(1, args.e2e_passes)
    t0 = time.perf_counter()
    for _ in range(passes):
        _, texts, prof = run()
    dt = (time.perf_counter() - t0) / passes
    same = same and texts == want
    keys_kept = int(pin["keys"].numel())
    del pin
    return {"Msites_per_s": round(args.sites / dt / 1e6, 2), "ms_per_run": round(dt * 1e3, 2),
            "h2d_bytes_per_run": prof["h2d_bytes"], "h2d_GBps_effective": round(prof["h2d_bytes"] / dt / 1e9, 2),
            "keys_in_piece": keys_kept, "chunks": prof["chunks"], "ms_h2d_device": round(prof["ms_h2d"], 2),
            "ms_call_device": round(prof["ms_call"], 2), "ms_finish": round(prof["ms_finish"], 2),
            "host_conversion_s": round(t_conv, 2), "runs": passes, "matches_resident": same,
            "how": "C-ABI pbg_stream_push_compact: reference-only tasks flagged in rmsq bit 31 without their keys "
                   "(pbf_compact of the pinned host batch, untimed: the feeder emits this form as it packs), then "
                   "the streamed run as above"}


def cli_rate(args) -> dict:
    """The drop-in command line on a real BAM: `popbam nucdiv|sfs|ld -f ref.fa -w 10 in.bam chr1`
    over a BAM of the first --cli-sample positions of the same synthetic genome
    (tests/ref_baseline.make_inputs, written natively):
      - as users run it: a fresh `bin/popbam` process per command (the native host binary,
        popbam_main.cpp: no interpreter, HIP init + context on a thread beside the feeder's
        walk), three runs per command, with the binary's own phase profile (POPBAM_PROFILE);
      - in-process (popbam_amd.cli.run, context and FASTA kept across commands) with its phases;
      - a fresh Python process (`python -m popbam_amd.cli`, no torch import) for comparison.
    stdout is compared with POPBAM's own on the same BAM, whose region-sharded run on every usable
    core is the all-core rate beside it (3 commands summed, as cpu_baseline)."""
    import subprocess
    import tempfile

    import ref_baseline
    from popbam_amd import cli
    L, n = args.cli_sample, args.samples
    t0 = time.perf_counter()
    d = ref_baseline.make_inputs(f"/tmp/popbam_refbase_v5_{args.seed:x}_{L}_{n}", args.seed, L, n)
    t_make = time.perf_counter() - t0
    win_kb = str(args.window // 1000)
    share = host_cpu_share()
    threads = int(os.environ.get("POPBAM_FEED_THREADS", share["cores"]))
    env = dict(os.environ, POPBAM_FEED_THREADS=str(threads))
    env.pop("WORLD_SIZE", None)
    res = {"sites": L, "samples": n, "feeder_threads": threads, "host": share,
           "bam_bytes": os.path.getsize(os.path.join(d, "in.bam")), "bam_write_s": round(t_make, 2), "commands": {}}
    texts = {}
    tot_in = tot_proc = tot_py = 0.0
    cwd = os.getcwd()
    runs = 3
    for c in ("nucdiv", "sfs", "ld"):
        argv = [c, "-f", "ref.fa", "-w", win_kb, "in.bam", "chr1"]
        # as users run it: a fresh native process per command
        proc_s, profs, same = [], [], True
        for _ in range(runs):
            with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as tf:
                pf = tf.name
            t0, w0 = time.perf_counter(), time.time()
            p = subprocess.run([os.path.join(REPO, "bin", "popbam"), *argv], cwd=d, capture_output=True,
                               env=dict(env, POPBAM_PROFILE=pf))
            proc_s.append(time.perf_counter() - t0)
            w1 = time.time()
            try:
                with open(pf) as f:
                    q = json.loads(f.read().splitlines()[-1])["popbam_profile"]
                # wall clock: spawn -> main, and _exit -> reaped by this process (kernel teardown)
                q["spawn_to_main_s"] = q.pop("main_wall_epoch_s", w0) - w0
                q["exit_to_reaped_s"] = w1 - q.pop("exit_wall_epoch_s", w1)
                for k2 in ("ms_stage", "ms_wait", "ms_h2d", "ms_call"):
                    q["gpu_" + k2] = q.get("gpu", {}).get(k2, 0.0)
                profs.append(q)
            except (OSError, ValueError, IndexError):
                profs.append({})
            os.unlink(pf)
            out_native = p.stdout.decode()
            same = same and p.returncode == 0
            texts.setdefault(c, out_native)
            same = same and out_native == texts[c]
        # in-process (context kept by cli across commands)
        os.environ["POPBAM_FEED_THREADS"] = str(threads)
        os.chdir(d)
        try:
            best = None
            for _ in range(2):   # the first run also builds the context
                t0 = time.perf_counter()
                text = cli.run(c, argv[1:])
                dt = time.perf_counter() - t0
                if best is None or dt < best[0]:
                    best = (dt, dict(cli.last_profile))
        finally:
            os.chdir(cwd)
        same_in = text == texts[c]
        t0 = time.perf_counter()
        pp = subprocess.run([sys.executable, "-m", "popbam_amd.cli", *argv], cwd=d, capture_output=True,
                            env=dict(env, PYTHONPATH=REPO))
        t_py = time.perf_counter() - t0
        pr = best[1]
        fe, gp = pr.get("feeder", {}), pr.get("gpu", {})
        mean_proc = sum(proc_s) / len(proc_s)
        keys = ("spawn_to_main_s", "parse_s", "fasta_s", "kstream_open_s", "hip_init_s", "pbg_create_s",
                "walk_during_gpu_init_s", "pieces_during_gpu_init", "gpu_join_wait_s", "stream_open_s", "first_push_s",
                "push_early_s", "push_calls_s", "keys_free_s", "walk_push_s", "gpu_ms_stage", "gpu_ms_wait", "gpu_ms_h2d", "gpu_ms_call", "finish_s",
                "run_s", "write_s", "exit_to_reaped_s")
        res["commands"][c] = {
            "process_s": [round(x, 3) for x in proc_s], "process_mean_s": round(mean_proc, 3),
            "process_identical": same and same_in and pp.returncode == 0 and pp.stdout.decode() == texts[c],
            "process_phases": {k: round(sum(q.get(k, 0.0) for q in profs) / max(1, len(profs)), 4) for k in keys},
            "process_phases_note": ("native binary: hip_init_s + pbg_create_s run on a thread while fasta, "
                                    "kstream_open and the walk proceed (walk_during_gpu_init_s: pieces taken "
                                    "meanwhile); gpu_join_wait_s is what the main thread then still waited; run_s = "
                                    "main's whole run, the rest of process_s is exec, library loading and exit"),
            "python_process_s": round(t_py, 3),
            "in_process_s": round(best[0], 3),
            "phases": {"fasta_s": round(pr.get("fasta_s", 0), 3), "context_s": round(pr.get("context_s", 0), 4),
                       "walk_and_push_s": round(pr.get("blocks_s", 0) - gp.get("ms_finish", 0) / 1e3, 3),
                       "feeder_thread_s": {"inflate": round(fe.get("t_inflate", 0), 3),
                                           "decode": round(fe.get("t_fetch", 0) - fe.get("t_inflate", 0), 3),
                                           "pileup_and_keys": round(fe.get("t_walk", 0), 3)},
                       "consumer_wait_for_feeder_s": round(fe.get("t_consumer_wait", 0), 3),
                       "host_staging_s": round(gp.get("ms_stage", 0) / 1e3, 3),
                       "h2d_device_s": round(gp.get("ms_h2d", 0) / 1e3, 4),
                       "call_device_s": round(gp.get("ms_call", 0) / 1e3, 4),
                       "finish_s": round(gp.get("ms_finish", 0) / 1e3, 4),
                       "h2d_bytes": gp.get("h2d_bytes", 0), "pieces": gp.get("pieces", 0),
                       "inflated_bytes": fe.get("bytes_inflated", 0)}}
        tot_in += best[0]
        tot_proc += mean_proc
        tot_py += t_py
    res["Msites_per_s_process"] = round(L / tot_proc / 1e6, 4)
    res["Msites_per_s_in_process"] = round(L / tot_in / 1e6, 4)
    res["Msites_per_s_python_process"] = round(L / tot_py / 1e6, 4)
    if ref_baseline.available():
        ac = popbam_all_cores(d, L, args.window)
        res["popbam_all_cores"] = {k: v for k, v in ac.items() if k != "texts"}
        res["x_process_over_popbam_all_cores"] = round(res["Msites_per_s_process"] / ac["Msites_per_s"], 2)
        res["x_in_process_over_popbam_all_cores"] = round(res["Msites_per_s_in_process"] / ac["Msites_per_s"], 2)
        res["identical_to_reference"] = all(ac["texts"][c] == texts[c] for c in texts)
    res["note"] = ("3 commands summed; process = mean of 3 fresh `bin/popbam` processes per command (native binary, "
                   "the drop-in as users run it); in-process = best of 2 runs of popbam_amd.cli.run (context kept "
                   "across commands); feeder_thread_s are summed over worker threads")
    return res


def parity_sampled_resident(args, ctx, hp, wins, contig: int) -> dict:
    """Checker (outside the timed region): --parity-windows windows of the timed configs[2] step,
    drawn at random, compared with the CPU oracle (tests/parity_sample.py): the rows of their
    positions bit for bit, their printed statistics byte for byte."""
    import parity_sample as ps
    rb = ctx.row_bytes
    idx = ps.pick(len(wins), args.parity_windows, args.seed ^ 0x5A5A)
    fields = hp.fields_for(hp.stats)
    picks = []
    for i in idx:
        a, b = wins[i]
        one = {}
        for k in fields:
            t = hp.out.t[k]
            per = t.numel() // max(1, len(wins))
            one[k] = t[i * per:(i + 1) * per].cpu().numpy()
        picks.append((contig, a, b, hp.rows[a * rb:b * rb].cpu().numpy(), one))
    t0 = time.perf_counter()
    r = ps.check_windows(ctx, ctx.params, picks, args.seed, args.depth, hp.stats)
    r["seconds"] = round(time.perf_counter() - t0, 2)
    return r


def parity_sampled_genome(args, ctx, gp, k: int) -> dict:
    """The same check on windows of a streamed configs[3] / [4] pass (rows of every chunk stay
    resident; window outputs per row group)."""
    import parity_sample as ps
    from popbam_amd import workload
    rb = ctx.row_bytes
    fields = workload.HotPath.fields_for(gp.stats)
    flat = []   # (segment, local window) in segment order = the order of gp.gstats' windows
    for si, w in enumerate(gp.win_lists):
        flat += [(si, j) for j in range(len(w))]
    where = []  # (group, index in group) in the same order
    for g, (_, _, _, nw, _, _) in enumerate(gp.gstats):
        where += [(g, j) for j in range(nw)]
    idx = ps.pick(len(flat), k, args.seed ^ 0x5A5A)
    picks = []
    for i in idx:
        si, j = flat[i]
        s = gp.segments[si]
        a, b = gp.win_lists[si][j]
        g, li = where[i]
        out, nw = gp.gstats[g][4], gp.gstats[g][3]
        one = {}
        for f in fields:
            t = out.t[f]
            per = t.numel() // max(1, nw)
            one[f] = t[li * per:(li + 1) * per].cpu().numpy()
        rows = gp.segment_rows(si)[a * rb:b * rb].cpu().numpy()
        picks.append((s.contig, s.beg + a, s.beg + b, rows, one))
    t0 = time.perf_counter()
    r = ps.check_windows(ctx, ctx.params, picks, args.seed, args.depth, gp.stats)
    r["seconds"] = round(time.perf_counter() - t0, 2)
    return r


def rows_crosscheck(torch, ctx, hp) -> dict:
    """Checker (outside the timed region), size-independent: the timed step's rows over the
    whole batch against the consensus-word call of the same batch (pbg_call_sites with words:
    call_sites_kernel runs errmod_cal + gl2cns on every task, none of the rows-only pipeline's
    shortcuts -- the reference-only test, uniform_ref, one_error_ref and their bound margins).
    Identical rows at every position are the full-size check of those shortcuts."""
    t0 = time.perf_counter()
    rows = hp.rows.clone()
    n = ctx.params.n_samples
    cb = torch.empty(hp.synth.n_sites * n, dtype=torch.int64, device="cuda")
    hp.call(cb=cb)
    torch.cuda.synchronize()
    ctx.sync_check()
    rb = ctx.row_bytes
    a, b = rows.view(-1, rb), hp.rows.view(-1, rb)
    ndiff = int((a != b).any(dim=1).sum().item())
    del cb
    hp.call()   # the rows-only rows back in place
    torch.cuda.synchronize()
    return {"identical": ndiff == 0, "positions": hp.synth.n_sites, "positions_differing": ndiff,
            "paths": "rows-only pipeline (scan shortcuts + queues) vs consensus-word call (full errmod per task)",
            "seconds": round(time.perf_counter() - t0, 2)}


def genome_rows_crosscheck(torch, ctx, gp, slot: int = 0) -> dict:
    """rows_crosscheck on one streamed chunk (chunk 0, generated into `slot`): the rows-only
    call and the consensus-word call of its whole batch, into scratch rows."""
    from popbam_amd import _lib
    t0 = time.perf_counter()
    si, p, L = gp.chunks[0]
    b = gp.buf[slot]
    pl = _lib.PbgPileup(L, p, b["ref"].data_ptr(), b["k"].data_ptr(), b["rmsq"].data_ptr(), b["block_off"].data_ptr(),
                        b["keys"].data_ptr())
    rb, n = ctx.row_bytes, ctx.params.n_samples
    fast = torch.zeros(L * rb, dtype=torch.uint8, device="cuda")
    full = torch.zeros_like(fast)
    cb = torch.empty(L * n, dtype=torch.int64, device="cuda")
    st = gp.call_stream.cuda_stream
    ctx.check(ctx.lib.pbg_call_sites(ctx.h, C.byref(pl), fast.data_ptr(), None, st), "pbg_call_sites")
    ctx.check(ctx.lib.pbg_call_sites(ctx.h, C.byref(pl), full.data_ptr(), cb.data_ptr(), st), "pbg_call_sites")
    gp.synchronize()
    ndiff = int((fast.view(-1, rb) != full.view(-1, rb)).any(dim=1).sum().item())
    del cb, fast, full
    return {"identical": ndiff == 0, "positions": L, "positions_differing": ndiff,
            "paths": "rows-only pipeline vs consensus-word call, chunk 0 of the pass",
            "seconds": round(time.perf_counter() - t0, 2)}


def zns_chain_floor(ld_snps, zns_ms: float | None = None) -> dict:
    """The ZnS sum's dependency floor (calc_zns, pop_ld.cpp:201-252): each window's r^2 values are
    added in the reference's pair order, one dependent f64 add after another, so the kernel cannot
    finish before its longest chain has.  window_zns_kernel pads each row of pairs to 16 (its
    rounds, zns_rounds in stats_kernel.hip); tools/ubench/fadd_chain.hip measures 7 cycles per
    dependent v_add_f64 with the operands in registers.  V is the window's S column (ns, which is
    the chain's variable-site count or one more)."""
    v = int(ld_snps.max().item()) if ld_snps.numel() else 0
    n = max(v - 1, 0)
    q, r = divmod(n, 16)
    rounds = (q + 1) * (8 * q + r)
    adds = 16 * rounds
    out = {"longest_chain_sites": v, "pairs": v * (v - 1) // 2, "adds_padded": adds,
           "floor_ms_at_7_cycles_2p4GHz": round(adds * 7 / 2.4e9 * 1e3, 4)}
    if zns_ms:
        out["kernel_ms"] = round(zns_ms, 4)
    return out


def max_over_ranks(dist, x: float) -> float:
    """The slowest rank's time (gloo, on the host)."""
    if not dist:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_genome(args, torch, dist, world, rank, binfo):
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
    xcheck = genome_rows_crosscheck(torch, ctx, gp) if (rank == 0 and args.parity_windows > 0) else None
    # the window statistics alone over the resident rows of the pass (HIP events on the call stream)
    win_ms = None
    if gp.stats:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        gp.stats_all()
        e0.record(gp.call_stream)
        for _ in range(3):
            gp.stats_all()
        e1.record(gp.call_stream)
        gp.synchronize()
        win_ms = e0.elapsed_time(e1) / 3
    pmc = pmc_traffic(args.config, {"contigs": args.contigs, "contig_len": args.contig_len, "samples": n,
                                    "depth": args.depth, "chunk": args.chunk, "world": world})
    traffic = pmc["kernels"]["call_scan_kernel"]["hbm_bytes"] if pmc else None
    call_traffic = sum(pmc["kernels"].get(k, {}).get("hbm_bytes", 0) for k in CALL_KERNELS) if pmc else None
    bpl = sb // max(1, chunks)
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
                         "traffic": traffic, "bytes_per_launch": bpl, "ms_per_launch": round(scan_ms, 4),
                         "traffic_ratio": round(traffic / bpl, 4) if traffic else None,
                         "traffic_split": traffic_split(traffic, scan_ms),
                         "call_stage_traffic": call_traffic,
                         "traffic_source": (f"{pmc['file']} (src_sha {pmc['src_sha']}, {pmc['source']}; mean over the "
                                            f"pass's chunk launches)" if pmc else
                                            "no PMC profile of this source tree (tools/pmc_traffic.sh)"),
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
            "window_stage": ({"ms_per_pass": round(win_ms, 3), "windows": gp.n_windows,
                              "row_bytes_per_pass": my_sites * ctx.row_bytes,
                              "GBps_rows": round(my_sites * ctx.row_bytes / (win_ms * 1e-3) / 1e9, 2),
                              "measured_on": "pbg_window_stats over the pass's resident rows, alone (3 passes, HIP "
                                             "events on the call stream)"} if win_ms else None),
            "note": "value includes the on-device generation of every pileup chunk (the input does not fit "
                    "HBM: ~1.8 TB of keys); call_stage is the call kernels alone (library HIP events)",
            "pass_mode": "overlapped (two streams)" if args.overlap else "serial (generate, then call, per chunk)",
        }
        out["cpu_baseline"] = cpu_baseline(args) if (world == 1 and args.cpu_sample > 0) else None
        if out["cpu_baseline"]:
            out["x_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
        if args.parity_windows > 0:
            ps = parity_sampled_genome(args, ctx, gp, max(4, args.parity_windows // (2 if args.config == 3 else 1)))
            out["parity_sampled"] = ps["ok"]
            out["parity_sample"] = ps
            out["rows_crosscheck"] = xcheck
        out["src_sha"] = source_hash()
        out["build"] = binfo
        print(json.dumps(out), flush=True)
    ctx.close()


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) run without a launcher: start N rank processes of this script, one per
    GPU, with the environment torch.distributed.run gives its workers (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT).  This process imports neither torch nor
    the library and never touches HIP; the ranks are children (subprocess), not an exec.  They
    inherit stdout, and only rank 0 prints the line.  Returns the first failing rank's status (the
    others are then terminated, so none is left waiting in a barrier), 0 when all succeed."""
    import socket
    import subprocess
    n = args.gpus
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0")
    argv = [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]
    procs = [subprocess.Popen(argv, env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad and rc == 0:
                rc = bad[0]
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    return 0 if rc == 0 else (rc if rc > 0 else 1)


def init_gloo(world: int):
    """gloo (host) process group for the timing barrier and the max over ranks: the data path
    has no collective, so RCCL is never initialised.  gloo announces its peer connections on
    stdout: they are kept off the one JSON line."""
    if world <= 1:
        return None
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def dry_run(args, world: int, rank: int):
    """--dry-run: the multi-rank launch and the shard plan without a GPU.  Each rank builds its
    shard (configs[2]: its own contig of --sites positions; configs[3]/[4]: genome.rank_plan),
    joins the same barrier + max-over-ranks timing as a real run, and rank 0 prints the line
    with `value` null, every rank's positions / windows, and whether the ranks' windows cover
    the workload exactly once."""
    dist = init_gloo(world)
    if os.environ.get("BENCH_DRY_FAIL_RANK") == str(rank):   # tests: a rank that dies before the barrier
        sys.exit(3)
    from popbam_amd import genome, workload
    if args.config == 2:
        mine = {"rank": rank, "sites": args.sites, "windows": len(workload.reference_windows(0, args.sites, args.window))}
        want_windows = mine["windows"] * world
    else:
        lengths = [args.contig_len] * args.contigs
        segs, _ = genome.rank_plan(args.config, lengths, world, rank, args.window, args.step)
        if args.config == 4:
            nw = sum(len(range(s.win_lo, s.win_hi, s.step)) for s in segs)
            want_windows = max(0, (args.contig_len - args.window) // args.step + 1)
        else:
            nw = sum(len(genome.contig_windows(args.contig_len, args.window, s.beg, s.end)) for s in segs)
            want_windows = sum(len(genome.contig_windows(L, args.window)) for L in lengths)
        mine = {"rank": rank, "sites": sum(s.end - s.beg for s in segs), "windows": nw, "segments": len(segs)}
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.perf_counter() - t0)
    ranks = [None] * world
    if dist:
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Msites/s", "n_gpus": world, "steps": 0,
                          "warmup": 0, "ms_per_step": None, "higher_is_better": True,
                          "scaling": "weak" if args.config == 2 else "strong", "vs_baseline": None, "dtype": "f64",
                          "data": "none (dry run: no GPU, no compute)", "dry_run": True,
                          "barrier_s": round(elapsed, 6), "config": {"workload": f"configs[{args.config}] shard plan",
                                                                     "parallelism": f"dp{world}"},
                          "ranks": ranks, "windows_covered": sum(r["windows"] for r in ranks) == want_windows}),
              flush=True)
    if dist:
        dist.destroy_process_group()


def build_info(allow_variant: bool) -> dict:
    """Which libpopbam_gpu.so this run measures (path and pbg_build_info(): 'product', 'bounds' or
    'experiment').  A non-product build (tools/variant.sh, a PBG_BOUNDS build; some give wrong
    results) is refused unless --allow-variant, and then the line carries its kind."""
    from popbam_amd import _lib
    kind = _lib.load().pbg_build_info().decode()
    info = {"kind": kind, "library": os.path.relpath(_lib.LIB_PATH, REPO) if _lib.LIB_PATH.startswith(REPO)
            else _lib.LIB_PATH}
    if kind != "product" and not allow_variant:
        sys.exit(f"bench.py: {info['library']} is a '{kind}' build, not the product (pass --allow-variant to "
                 "measure it anyway; the line then records build.kind)")
    return info


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {args.gpus}: they must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run(args, world, rank)
        return
    import torch

    dist = None
    binfo = build_info(args.allow_variant)
    if world > 1:
        # one rank per GPU; more ranks than GPUs (a rehearsal on a smaller box) share them
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist = init_gloo(world)
    else:
        torch.cuda.set_device(0)

    if args.config in (3, 4):
        bench_genome(args, torch, dist, world, rank, binfo)
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

    # per-launch HBM traffic from rocprofv3 PMC counters of this source tree (else null)
    pmc = pmc_traffic(2, {"sites": args.sites, "samples": n, "depth": args.depth, "pieces": len(pts) - 1})
    traffic = pmc["kernels"]["call_scan_kernel"]["hbm_bytes"] if pmc else None
    call_traffic = sum(pmc["kernels"].get(k, {}).get("hbm_bytes", 0) for k in CALL_KERNELS) if pmc else None

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
                         "traffic_ratio": round(traffic / scan_bytes_launch, 4) if traffic else None,
                         "traffic_split": traffic_split(traffic, scan_ms),
                         "traffic_source": (f"{pmc['file']} (src_sha {pmc['src_sha']}, {pmc['source']})" if pmc else
                                            "no PMC profile of this source tree (tools/pmc_traffic.sh)"),
                         "bytes_basis": "SURVEY 8(d): sum over (position, sample) of 2k+5, +1 +row_bytes per position",
                         "layout_bytes_per_launch": layout_bytes,
                         "frac_layout": round(layout_bytes * args.steps / (kt.value * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "call_stage": {"ms_serial": round(call_ms, 4), "ms_library_events": round(call_lib_ms, 4),
                           "bytes": call_bytes, "GBps": round(call_bytes / (call_lib_ms * 1e-3) / 1e9, 2),
                           "frac": round(call_bytes / (call_lib_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "kernels": "call_scan + call_slow + call_deepq + call_overflow + call_fold",
                           "traffic": call_traffic,
                           "traffic_ratio": round(call_traffic / call_bytes, 4) if call_traffic else None},
            "window_stats": {"ms_serial": round(stats_ms, 4), "rows_bytes": stats_bytes,
                             "GBps": round(stats_bytes / (stats_ms * 1e-3) / 1e9, 2),
                             "Msites_per_s_stats_only": round(args.sites / (stats_ms * 1e-3) / 1e6, 2),
                             "zns_chain": zns_chain_floor(hp.out.t["ld_snps"])},
        }
        if world == 1:
            out["pcie_inclusive"] = pcie_rate(torch, layout_bytes - args.sites * n, elapsed / args.steps, args.sites)
            if args.e2e_chunk >= 0 and args.cpu_sample > 0:   # --cpu-sample 0 (profiling runs) skips the extras
                out["end_to_end"] = end_to_end(args, torch, ctx, hp, wins)
            if args.cli_sample > 0 and args.cpu_sample > 0:
                out["cli"] = cli_rate(args)
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(args)
        else:
            out["cpu_baseline"] = None
        if args.parity_windows > 0:
            ps = parity_sampled_resident(args, ctx, hp, wins, rank)
            out["parity_sampled"] = ps["ok"]
            out["parity_sample"] = ps
            out["rows_crosscheck"] = rows_crosscheck(torch, ctx, hp)
        out["src_sha"] = source_hash()
        out["build"] = binfo
        print(json.dumps(out), flush=True)
    ctx.check(ctx.lib.pbg_set_kernel_timing(ctx.h, 0), "pbg_set_kernel_timing")
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
