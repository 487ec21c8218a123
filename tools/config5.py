"""Config 5 timing: 16 right-hand sides at the config-3 geometry,
mode 0 -- the mixed-precision multi-RHS solver (aniso_amd/solve.py) with the fp32
MFMA inner operator, the same solver with the fp64 inner operator (the previous
round's), and 16 fp64 single-RHS device GMRES solves; plus the fp32 and fp64
16-RHS operator times (fp64: two 8-RHS VALU batches and the fp64 MFMA operator).  Prints one JSON line."""
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
gmres_mixed(a, B, tol=1e-12)  # warm-up (also builds the fp32 caches)
torch.cuda.synchronize()
res = {}
for name, f32, f64m in (("mixed_fp32_mfma", True, True), ("mixed_fp32_mfma_valu_refinement", True, False),
                        ("mixed_fp64_inner", False, False)):
    t0 = time.perf_counter()
    X, outer, inner, rel = gmres_mixed(a, B, tol=1e-12, m=40, inner_tol=1e-6, fp32_op=f32, fp64_mfma=f64m)
    torch.cuda.synchronize()
    res[name] = {"s": round(time.perf_counter() - t0, 4), "outer": outer, "inner_iterations": inner,
                 "final_rel_residual_max": float(rel.max())}
    if f32:
        Xf = X.cpu().numpy()
# operator times: 16 right-hand sides, fp32 MFMA vs two fp64 8-RHS batched applies
X32 = torch.rand(a.N, 16, device="cuda", dtype=torch.float32)
Y32 = torch.empty_like(X32)
W = torch.empty_like(B)
for _ in range(3):
    a.forward_f32_dev(X32, Y32)
a.set_timing(True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    a.forward_f32_dev(X32, Y32)
torch.cuda.synchronize()
t32 = (time.perf_counter() - t0) / 20
st32 = a.stage_times()
a.set_timing(False)
from aniso_amd.solve import forward_block  # noqa: E402

for _ in range(2):
    forward_block(a, B, W)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    forward_block(a, B, W)
torch.cuda.synchronize()
t64 = (time.perf_counter() - t0) / 10
from aniso_amd.solve import forward16  # noqa: E402

perm = torch.tensor(a.tree_perm(), device="cuda", dtype=torch.int64)
for _ in range(2):
    forward16(a, B, W, perm)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    forward16(a, B, W, perm)
torch.cuda.synchronize()
t64m = (time.perf_counter() - t0) / 10
t0 = time.perf_counter()
errs, its_ref = [], []
for s in range(k):
    its, x, hist, fr = a.gmres(Q[s], m=80, maxit=400, tol=1e-12)
    its_ref.append(its)
    errs.append(float(np.linalg.norm(Xf[s] - x) / np.linalg.norm(x)))
t_ref = time.perf_counter() - t0
print(json.dumps({"config": f"configs[4]: sz={sz} (N={a.N}), d=1, ns=10, mode 0, 16 RHS", **res,
                  "op16_fp32_mfma_ms": round(1e3 * t32, 4), "op16_fp32_stage_ms": {kk: round(v, 4) for kk, v in st32.items()},
                  "op16_fp64_ms": round(1e3 * t64, 4), "op16_fp64_mfma_ms_incl_transposes": round(1e3 * t64m, 4),
                  "fp32_cache_bytes": a.stats()["f32_cache_bytes"],
                  "fp64_single_rhs_s": round(t_ref, 4), "fp64_iterations": its_ref,
                  "rel_err_vs_fp64_max": max(errs)}))
