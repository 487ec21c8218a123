"""Cost of the stage timers (HIP events between the apply's launches) on the 1M-point
block matvec: one handle, repetitions with the timers off, on (level 1) and at the
roofline spans only (level 2) interleaved.
usage: timing_overhead.py [--reps R] [--steps S]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--steps", type=int, default=30)
args = ap.parse_args()
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)
levels = {"off": 0, "on": 1, "roofline": 2}  # aniso_set_timing levels
res = {k: [] for k in levels}
for rep in range(args.reps):
    for mode, level in levels.items():
        op.set_timing(level)
        for _ in range(3):
            op.block_op_dev(2, x, y, tree=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            op.block_op_dev(2, x, y, tree=True)
        torch.cuda.synchronize()
        res[mode].append(round(1e3 * (time.perf_counter() - t0) / args.steps, 4))
        op.set_timing(False)
op.sync()
med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
print(json.dumps({"ms": res, "median_ms": med, "overhead": round(med["on"] / med["off"] - 1, 4),
                  "overhead_roofline": round(med["roofline"] / med["off"] - 1, 4)}), flush=True)
