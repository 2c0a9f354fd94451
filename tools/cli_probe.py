"""The drop-in command line alone (bench.py's `cli` leg and the all-core POPBAM figure), without
the GPU benchmark steps: `python tools/cli_probe.py [--cli-sample N]` prints one JSON object."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cli-sample", type=int, default=5_000_000)
ap.add_argument("--samples", type=int, default=12)
ap.add_argument("--window", type=int, default=10_000)
ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xC0FFEE02)
a = ap.parse_args()
import torch  # noqa: E402,F401  (the in-process leg shares the process with torch, as in bench.py)
print(json.dumps({"host": bench.host_cpu_share(), "cli": bench.cli_rate(a)}), flush=True)
