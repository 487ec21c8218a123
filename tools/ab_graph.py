"""Block matvec at 1M points: eager launches vs one captured HIP graph per step
(torch.cuda.CUDAGraph around aniso_block_op_dev, both its streams), and the
graph's output vs the eager one.  usage: ab_graph.py [steps] [world rank]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x0 = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x0[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
a, b = x0.clone(), torch.zeros_like(x0)


def eager(n):
    global a, b
    for _ in range(n):
        op.block_op_dev(2, a, b, tree=True)
        a, b = b, a


res = {}
eager(3)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    eager(steps)
    torch.cuda.synchronize()
    res[f"eager_ms_{rep}"] = round(1e3 * (time.perf_counter() - t0) / steps, 4)
ref = torch.zeros_like(x0)
op.block_op_dev(2, x0, ref, tree=True)
# two graphs: a -> b and b -> a
ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    op.block_op_dev(2, a, b, tree=True)
    op.block_op_dev(2, b, a, tree=True)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(ga):
    op.block_op_dev(2, a, b, tree=True)
with torch.cuda.graph(gb):
    op.block_op_dev(2, b, a, tree=True)
a.copy_(x0)
ga.replay()
torch.cuda.synchronize()
res["graph_vs_eager_max_abs"] = float((b - ref).abs().max())
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps // 2):
        ga.replay()
        gb.replay()
    torch.cuda.synchronize()
    res[f"graph_ms_{rep}"] = round(1e3 * (time.perf_counter() - t0) / (2 * (steps // 2)), 4)
print(json.dumps(res))
