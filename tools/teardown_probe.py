"""Exit -> reaped time of HIP processes by allocation size (tools/ubench/exit_teardown): what a
fresh process pays after its last output, as a function of device / pinned memory held."""
import json
import os
import subprocess
import time

B = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench", "exit_teardown")
out = []
import sys
CASES = ((0, 0, 1, 0, 0), (64, 0, 1, 0, 0), (1024, 0, 1, 0, 0), (0, 64, 1, 0, 0), (0, 256, 1, 0, 0), (0, 1024, 1, 0, 0),
         (64, 64, 32, 0, 0), (0, 0, 1, 0, 0))
if len(sys.argv) > 1 and sys.argv[1] == "host":
    CASES = ((64, 64, 1, 0, 0), (64, 64, 1, 1500, 0), (64, 64, 1, 1500, 1), (64, 64, 1, 400, 1))
for dev, pin, ch, hmb, fr in CASES:
    for _ in range(3):
        t0 = time.time()
        r = subprocess.run([B, str(dev), str(pin), str(ch), str(hmb), str(fr)], capture_output=True, text=True)
        t1 = time.time()
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out.append({"dev_mb": dev, "pin_mb": pin, "chunks": ch, "host_mb": hmb, "free": fr, "proc_s": round(t1 - t0, 4),
                    "init_s": d["init_s"], "alloc_s": d["alloc_s"], "free_s": d.get("free_s"),
                    "exit_to_reaped_s": round(t1 - d["exit_epoch"], 4)})
        print(json.dumps(out[-1]), flush=True)
