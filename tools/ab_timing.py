"""Block matvec wall time at 1M points with and without the per-stage HIP events
(aniso_set_timing), to price the events bench.py records in its timed region.
usage: ab_timing.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)


def run(timing):
    global x, y
    op.set_timing(timing)
    for _ in range(3):
        op.block_op_dev(2, x, y, tree=True)
        x, y = y, x
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        op.block_op_dev(2, x, y, tree=True)
        x, y = y, x
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = op.stage_times() if timing else {}
    op.set_timing(False)
    return 1e3 * el / steps, st


res = {}
for rep in range(2):
    for tm in (False, True):
        ms, st = run(tm)
        res[f"{'events' if tm else 'no_events'}_{rep}"] = round(ms, 4)
print(json.dumps(res))
