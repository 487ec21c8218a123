"""Per-rank block-matvec time of one shard (no collective): what one GPU of an
N-GPU strong-scaling run computes per step.  usage: shard_time.py WORLD [RANK]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from aniso_amd import dist as adist  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
ranges = adist.shard_ranges(op, world)
op.set_shard(rank, world)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
L = adist.pad_len(ranges)
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
slab = torch.zeros(5, L, dtype=torch.float64, device="cuda")
for _ in range(3):
    op.block_op_dev(2, x, slab, tree=True)
op.set_timing(True)
torch.cuda.synchronize()
t0 = time.perf_counter()
steps = 20
for _ in range(steps):
    op.block_op_dev(2, x, slab, tree=True)
torch.cuda.synchronize()
ms = 1e3 * (time.perf_counter() - t0) / steps
st = op.stats()
print(json.dumps({"world": world, "rank": rank, "ms_per_apply": round(ms, 4),
                  "stage_ms": {k: round(v, 4) for k, v in op.stage_times().items()},
                  "m2l_clusters": st["hm_clusters"], "m2l_targets": st["m2l_targets"], "leaves": st["leaves"]}))
