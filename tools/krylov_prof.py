"""The Krylov legs of bench.py at 1M points, twice each in one process: aniso.m's block
solve (aniso_block_solve_dev, gmres(A, rhs, 400, 1e-11, 400)) and the GMRES leg
(gmres_dist on the library's Arnoldi, 30 steps, tol 0), wall times per call; run it
under rocprofv3 --kernel-trace --stats for the per-kernel split.
usage: krylov_prof.py [sz] [gmres steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from aniso_amd.solve import gmres_dist  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
op = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
charge = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
charge[0] = torch.tensor(gaussian(xy), device="cuda")
rhs = torch.zeros_like(charge)
op.block_op_dev(0, charge, rhs)
x = charge.clone()
y = torch.zeros_like(x)
for _ in range(5):
    op.block_op_dev(2, x, y, tree=True)
    x, y = y, x
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    op.block_op_dev(2, x, y, tree=True)
    x, y = y, x
torch.cuda.synchronize()
mv = (time.perf_counter() - t0) / 20
print(json.dumps({"matvec_ms": round(1e3 * mv, 4)}), flush=True)
for k in range(2):
    u = torch.zeros_like(charge)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its, _, rel = op.block_solve_dev(rhs, u, 400, 1e-11, 400)
    el = time.perf_counter() - t0
    print(json.dumps({"solve": k, "iterations": its, "relres": rel, "seconds": round(el, 4),
                      "ms_per_iteration": round(1e3 * el / max(abs(its), 1), 4),
                      "non_matvec_ms_per_iteration": round(1e3 * (el - (abs(its) + 1) * mv) / max(abs(its), 1), 4)}),
          flush=True)
gb = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
gb[0] = torch.tensor(gaussian(xy), device="cuda")[perm]


def gapply(a, b):
    op.block_op_dev(2, a, b, tree=True)


for k in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, its, rel = gmres_dist(gapply, gb, restart=steps, tol=0.0, maxit=1, kry=op)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"gmres": k, "steps": steps, "ms_per_step": round(1e3 * el / steps, 4),
                      "non_matvec_ms_per_step": round(1e3 * (el - (steps + 1) * mv) / steps, 4)}), flush=True)
