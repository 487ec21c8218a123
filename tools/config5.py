"""Config 5 timing: 16 right-hand sides at the config-3 geometry,
mode 0 -- the mixed-precision multi-RHS solver (aniso_amd/solve.py) against 16 fp64
single-RHS device GMRES solves.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from aniso_amd.solve import config5_charges, gmres_mixed, rhs_block  # noqa: E402
from bench import main_coeffs  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
xy = a.getNodes()
a.setCoeff(*main_coeffs(xy))
a.cache(0)
k = 16
Q = np.stack([config5_charges(xy, s) for s in range(k)])
Qd = torch.tensor(Q, device="cuda")
B = rhs_block(a, Qd)
gmres_mixed(a, B[:8], tol=1e-12)  # warm-up
torch.cuda.synchronize()
t0 = time.perf_counter()
X, outer, inner, rel = gmres_mixed(a, B, tol=1e-12, m=40, inner_tol=1e-6)
torch.cuda.synchronize()
t_mixed = time.perf_counter() - t0
t0 = time.perf_counter()
errs, its_ref = [], []
Xh = X.cpu().numpy()
for s in range(k):
    its, x, hist, fr = a.gmres(Q[s], m=80, maxit=400, tol=1e-12)
    its_ref.append(its)
    errs.append(float(np.linalg.norm(Xh[s] - x) / np.linalg.norm(x)))
t_ref = time.perf_counter() - t0
print(json.dumps({"config": f"configs[4]: sz={sz} (N={a.N}), d=1, ns=10, mode 0, 16 RHS",
                  "mixed_s": round(t_mixed, 4), "outer": outer, "inner_iterations": inner,
                  "final_rel_residual_max": float(rel.max()), "fp64_single_rhs_s": round(t_ref, 4),
                  "fp64_iterations": its_ref, "rel_err_vs_fp64_max": max(errs)}))
