"""Iteration counts of aniso_block_solve on small systems (probe for test sizing)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch, aniso_amd
from conftest import gaussian_charge, main_coeffs, rough_coeffs  # noqa: E402
for sz, kind, g in [(32, "main", 0.8), (24, "rough", 0.8), (32, "rough", 0.95), (16, "rough", 0.95)]:
    a = aniso_amd.Aniso(sz, 1, 5, g, 10, 4, 20)
    xy = a.getNodes()
    cf = main_coeffs(xy) if kind == "main" else rough_coeffs(xy, 3)
    a.setCoeff(*cf)
    for m in range(9):
        a.cache(m)
    rhs = np.random.default_rng(1).uniform(-1, 1, 5 * a.N)
    for tol in (1e-11, 1e-13, 1e-14):
        its, u, hist, rr = a.block_solve(rhs, 200, tol, 1)
        print(sz, kind, g, tol, its, rr, flush=True)
