"""The fp64 16-right-hand-side MFMA operator alone (f64op.hip, 1M points by default):
main.cpp's forward operator on 16 right-hand sides, timed against the same operator as
two 8-right-hand-side batches of the VALU block apply (aniso_amd.solve.forward_block,
what config 5's fp64 refinement used before), and the largest column difference.
usage: f64op_bench.py [sz] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from aniso_amd.solve import forward_block, forward16  # noqa: E402
from bench import main_coeffs  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
a.setCoeff(*main_coeffs(a.getNodes()))
a.cache(0)
perm = torch.tensor(a.tree_perm(), device="cuda", dtype=torch.int64)
X = torch.rand(16, a.N, device="cuda", dtype=torch.float64)
W1, W2 = torch.empty_like(X), torch.empty_like(X)
X16 = X[:, perm].t().contiguous()
Y16 = torch.empty_like(X16)


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


a.set_timing(True)
ms_mfma = timed(lambda: a.forward16_f64_dev(X16, Y16))
st = a.stage_times()
a.set_timing(False)
ms_valu = timed(lambda: forward_block(a, X, W1))
forward16(a, X, W2, perm)
torch.cuda.synchronize()
err = float(torch.linalg.norm(W2 - W1) / torch.linalg.norm(W1))
print(json.dumps({"N": a.N, "rhs": 16, "fp64_mfma_ms_per_apply": round(ms_mfma, 4),
                  "fp64_valu_two_batches_ms": round(ms_valu, 4), "speedup": round(ms_valu / ms_mfma, 2),
                  "rel_diff_vs_valu": err, "stage_ms": {k: round(v, 4) for k, v in st.items()}}), flush=True)
