#!/usr/bin/env python3
"""Diagnostic: generate configs[3] chunks one at a time (synchronously) and check each chunk's
block_off against its k[] block sums; then run the double-buffered pass synchronously
(POPBAM_GENOME_SYNC) and asynchronously, reporting which mode trips pbg_check."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from popbam_amd import _lib, genome, workload  # noqa: E402

n, chunk = 24, 1 << 25
ctx = _lib.Context(workload.default_params(n), 0)
lengths = [125_000_000] * int(os.environ.get("CONTIGS", "2"))
segs = genome.plan_genome(lengths, 1, 10_000)[0]
stats = int(os.environ.get("STATS", "0"))
gp = genome.GenomePass(ctx, segs, 0xC0FFEE04, 10, 10_000, stats, chunk)
if os.environ.get("SKIP_GEN"):
    gp.chunks_all = gp.chunks
bad = 0
for c in range(0 if os.environ.get("SKIP_GEN") else len(gp.chunks)):
    gp._generate(c, 0)
    torch.cuda.synchronize()
    L = gp.chunks[c][2]
    nb = (L + 63) // 64
    b = gp.buf[0]
    k = b["k"][:L * n].to(torch.int64)
    pad = nb * 64 * n - L * n
    if pad:
        k = torch.cat([k, torch.zeros(pad, dtype=torch.int64, device=k.device)])
    sums = k.view(nb, 64 * n).sum(1)
    bo = b["block_off"][:nb + 1]
    diff = bo[1:] - bo[:-1]
    mism = int((sums != diff).sum())
    print(f"chunk {c} L={L} keys={int(bo[nb])} cap={gp.keys_cap} mismatching blocks={mism} first_off={int(bo[0])}", flush=True)
    bad += mism
ctx.check(ctx.lib.pbg_check(ctx.h, None), "pbg_check after generation")
print("generation check:", "OK" if bad == 0 else f"{bad} bad blocks", flush=True)
for mode in os.environ.get("MODES", "sync,async").split(","):
    try:
        if mode == "sync":
            for c in range(len(gp.chunks)):
                gp._generate(c, c & 1)
                torch.cuda.synchronize()
                gp._call(c, c & 1)
                torch.cuda.synchronize()
                ctx.check(ctx.lib.pbg_check(ctx.h, None), f"chunk {c}")
        elif mode == "async":
            gp.call_all()
            gp.synchronize()
        else:   # the bench's pass: calls, then statistics
            gp.run()
            gp.synchronize()
        print(mode, "OK", flush=True)
    except Exception as e:  # noqa: BLE001
        print(mode, "FAILED", e, flush=True)
ctx.close()
