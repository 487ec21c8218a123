"""Per-task phase timeline of the down pass (k_down_tier) of one block matvec, from a
library built with -DANISO_DOWN_TRACE (tools/build_variant.sh dt "-DANISO_DOWN_TRACE=1";
run with ANISO_LIB=build/ab_dt/libaniso_mi355x.so).  usage: down_trace.py [WORLD]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
if world > 1:
    op.set_shard(0, world)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)
if world > 1:
    op.comm_init_loopback()
for _ in range(4):
    if world > 1:
        op.block_op_sharded_dev(2, x, y)
    else:
        op.block_op_dev(2, x, y, tree=True)
torch.cuda.synchronize()
ntask = 16384
buf = (ctypes.c_longlong * (ntask * 6))()
assert aniso_amd.lib().aniso_debug_down_trace(buf, ntask) == 0
tr = np.frombuffer(buf, dtype=np.int64).reshape(ntask, 6)
tr = tr[tr[:, 0] > 0]
t0 = tr[:, 0].min()
us = (tr[:, :5] - t0) / 100.0
ph = np.diff(us, axis=1)  # loads, chain, levels, points
rep = {"world": world, "tasks": int(len(tr)), "launch_us": round(float(us[:, 4].max()), 2),
       "phase_us_p50": [round(float(v), 2) for v in np.percentile(ph, 50, axis=0)],
       "phase_us_p90": [round(float(v), 2) for v in np.percentile(ph, 90, axis=0)],
       "task_us": {q: round(float(np.percentile(us[:, 4] - us[:, 0], p)), 2) for q, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))},
       "start_us": {q: round(float(np.percentile(us[:, 0], p)), 2) for q, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))}}
mid = np.percentile(us[:, 4], 50)
rep["resident_at_p50_end"] = int(((us[:, 0] <= mid) & (us[:, 4] >= mid)).sum())
print(json.dumps(rep), flush=True)
