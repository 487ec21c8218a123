"""Per-rank compute of the sharded forward operator, simulated on one GPU.

For nranks in 1, 2, 4, 8 the operator is sharded (aniso_set_shard) and one rank's
tree-order forward operator is timed alone (no collective): what one GPU of an
N-GPU run computes per matvec.  usage: python tools/shard_sim.py [rank ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import gaussian, main_coeffs  # noqa: E402

ranks = [int(a) for a in sys.argv[1:]] or [0]
torch.cuda.set_device(0)
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
ss, st = main_coeffs(xy)
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
x = torch.tensor(gaussian(xy), device="cuda")[perm].contiguous()
for n in (1, 2, 4, 8):
    for r in ranks:
        if r >= n:
            continue
        op.set_shard(r, n)
        op.setCoeff(ss, st)
        op.cache(0)
        y = torch.zeros(op.N, dtype=torch.float64, device="cuda")
        for _ in range(3):
            op.forward_tree_dev(x, y)
        op.set_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            op.forward_tree_dev(x, y)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        st_ = op.stage_times()
        op.set_timing(False)
        s = op.stats()
        print(json.dumps({"nranks": n, "rank": r, "ms_per_matvec": round(dt * 1e3, 4), "shard": op.shard(),
                          "stored_m2l": s["stored_m2l"], "stage_ms": {k: round(v, 4) for k, v in st_.items()}}),
              flush=True)
