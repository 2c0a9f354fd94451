"""Exit -> reaped time of HIP processes by allocation size (tools/ubench/exit_teardown): what a
fresh process pays after its last output, as a function of device / pinned memory held."""
import json
import os
import subprocess
import time

B = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ubench", "exit_teardown")
out = []
for dev, pin, ch in ((0, 0, 1), (64, 0, 1), (1024, 0, 1), (0, 64, 1), (0, 256, 1), (0, 1024, 1), (64, 64, 32),
                     (0, 0, 1)):
    for _ in range(3):
        t0 = time.time()
        r = subprocess.run([B, str(dev), str(pin), str(ch)], capture_output=True, text=True)
        t1 = time.time()
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out.append({"dev_mb": dev, "pin_mb": pin, "chunks": ch, "proc_s": round(t1 - t0, 4), "init_s": d["init_s"],
                    "alloc_s": d["alloc_s"], "exit_to_reaped_s": round(t1 - d["exit_epoch"], 4)})
        print(json.dumps(out[-1]), flush=True)
