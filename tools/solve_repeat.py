"""aniso.m's block solve (aniso_block_solve_dev) run three times in one process at 1M
points: the first call's wall time includes the 401 x 5 x N Krylov basis allocation,
the later ones show whether that (not the iterations) moves bench.py's block_solve.
usage: solve_repeat.py [sz]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
op = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
charge = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
charge[0] = torch.tensor(gaussian(xy), device="cuda")
rhs = torch.zeros_like(charge)
op.block_op_dev(0, charge, rhs)
for k in range(3):
    u = torch.zeros_like(charge)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its, _, rel = op.block_solve_dev(rhs, u, 400, 1e-11, 400)
    el = time.perf_counter() - t0
    print(json.dumps({"call": k, "iterations": its, "relres": rel, "seconds": round(el, 4),
                      "ms_per_iteration": round(1e3 * el / max(abs(its), 1), 4)}), flush=True)
