"""The deterministic block matvec's distance from the default one:
relative 2-norm and max-entry differences at BASELINE's 1M-point configuration and at
inputs scaled by 1e+-150, plus repeat-equality.  Development tool (one JSON line)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
import aniso_amd  # noqa: E402
from conftest import rough_coeffs  # noqa: E402

a = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = a.getNodes()
a.setCoeff(*rough_coeffs(xy, 2))
for m in range(9):
    a.cache(m)
out = {}
U0 = torch.tensor(np.random.default_rng(8).uniform(-1, 1, (5, a.N)), device="cuda")
for scale in (1.0, 1e150, 1e-150):
    U = scale * U0
    a.set_deterministic(False)
    ref, ref2 = torch.zeros_like(U), torch.zeros_like(U)
    a.block_op_dev(2, U, ref, tree=True)
    a.block_op_dev(2, U, ref2, tree=True)
    a.set_deterministic(True)
    o1, o2 = torch.zeros_like(U), torch.zeros_like(U)
    a.block_op_dev(2, U, o1, tree=True)
    a.block_op_dev(2, U, o2, tree=True)
    torch.cuda.synchronize()
    out[str(scale)] = {
        "det_vs_default_rel2": float(torch.linalg.norm(o1 - ref) / torch.linalg.norm(ref)),
        "det_vs_default_relmax": float((o1 - ref).abs().max() / ref.abs().max()),
        "default_repeat_rel2": float(torch.linalg.norm(ref2 - ref) / torch.linalg.norm(ref)),
        "det_repeat_bitwise": bool(torch.equal(o1, o2)),
    }
print(json.dumps(out))
