"""Chained block matvecs at 1M points for a kernel trace (rocprofv3 --kernel-trace):
stage events off unless argv[2] == 'events'.  usage: trace_steps.py [steps] [events]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)
op.set_timing(len(sys.argv) > 2 and sys.argv[2] == "events")
for _ in range(steps):
    op.block_op_dev(2, x, y, tree=True)
    x, y = y, x
torch.cuda.synchronize()
print("done")
