"""Per-block timeline of the fused top-of-tree + clustered M2L launch (k_top_m2l_hc)
of one shard's block matvec: when each up task and cluster started, finished waiting
and ended, what it waited for and how many blocks it read.  Run with
ANISO_TOP_TRACE=1.  usage: top_trace.py WORLD RANK OUT.npy"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

native = "--native" in sys.argv  # the library's one-call matvec over a loopback communicator
argv = [a for a in sys.argv[1:] if not a.startswith("--")]
world, rank = int(argv[0]), int(argv[1])
out = argv[2] if len(argv) > 2 else None
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.set_shard(rank, world)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
b, e = op.shard()
ex = op.shard_exchange(5)
C, R = ex["root_chunk"], ex["root_record"]
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)
send = torch.zeros(max(C * R, 1), dtype=torch.float64, device="cuda")
recv = torch.zeros(world * max(C * R, 1), dtype=torch.float64, device="cuda")
if native and world > 1:
    op.comm_init_loopback()


def step():
    if world == 1:
        op.block_op_dev(2, x, y, tree=True)
        return
    if native:
        op.block_op_sharded_dev(2, x, y)
        return
    op.block_op_begin_dev(2, x, y[:, b:e], send)
    recv[rank * C * R:(rank + 1) * C * R].copy_(send[: C * R])
    op.block_op_end_dev(2, x, y[:, b:e], recv, world)


runs = []
for it in range(6):
    step()
    torch.cuda.synchronize()
    if it >= 3:
        runs.append(op.top_trace())
tr = runs[-1]
if out:
    np.save(out, np.stack(runs))
t0 = tr[:, 0].min()
us = lambda v: (v - t0) / 100.0  # noqa: E731  (100 MHz ticks -> microseconds)
nr = tr[tr[:, 4] == -99]  # near-field groups riding at the end of the launch (ANISO_NEAR_IN_TOP=1)
up = tr[(tr[:, 4] < 0) & (tr[:, 4] != -99)]
cl = tr[tr[:, 4] >= 0]
rep = {"world": world, "rank": rank, "launch_us": [round(float((r[:, 2].max() - r[:, 0].min()) / 100.0), 2) for r in runs],
       "blocks": int(tr.shape[0]), "up_blocks": int(up.shape[0]), "clusters": int(cl.shape[0])}
tiers = {}
for k in sorted(set((-up[:, 4]).tolist())):
    u = up[-up[:, 4] == k]
    tiers[int(k)] = {"n": int(u.shape[0]), "first_start": round(float(us(u[:, 0].min())), 2),
                     "last_waited": round(float(us(u[:, 1].max())), 2), "last_end": round(float(us(u[:, 2].max())), 2),
                     "mean_run_us": round(float((u[:, 2] - u[:, 1]).mean() / 100.0), 2)}
rep["tiers"] = tiers
if len(nr):
    rep["near_groups"] = {"n": int(len(nr)), "start_us": {q: round(float(np.percentile(us(nr[:, 0]), p)), 2) for q, p in
                                                      (("p0", 0), ("p50", 50), ("p100", 100))},
                          "run_us_p50": round(float(np.percentile((nr[:, 2] - nr[:, 1]) / 100.0, 50)), 2),
                          "end_us_max": round(float(us(nr[:, 2]).max()), 2)}
dur = (cl[:, 2] - cl[:, 1]) / 100.0
wait = (cl[:, 1] - cl[:, 0]) / 100.0
reads = cl[:, 7]
rep["cluster_run_us"] = {q: round(float(np.percentile(dur, p)), 2) for q, p in
                         (("p0", 0), ("p10", 10), ("p50", 50), ("p90", 90), ("p100", 100))}
rep["cluster_start_us"] = {q: round(float(np.percentile(us(cl[:, 0]), p)), 2) for q, p in
                           (("p0", 0), ("p50", 50), ("p90", 90), ("p100", 100))}
rep["cluster_end_us"] = {q: round(float(np.percentile(us(cl[:, 2]), p)), 2) for q, p in
                         (("p10", 10), ("p50", 50), ("p90", 90), ("p100", 100))}
rep["reads"] = {"total": int(reads.sum()), "max": int(reads.max()), "mean": round(float(reads.mean()), 1)}
rep["ns_per_read"] = round(float(1e3 * dur.sum() / max(reads.sum(), 1)), 1)
w = cl[:, 5] > 0
rep["waiting_clusters"] = {"n": int(w.sum()), "wait_us_max": round(float(wait[w].max()), 2) if w.any() else 0.0,
                           "end_us_max": round(float(us(cl[w, 2]).max()), 2) if w.any() else 0.0}
# the last clusters to finish
last = np.argsort(cl[:, 2])[-12:]
rep["last"] = [{"cid": int(cl[i, 4]), "wait_tier": int(cl[i, 5]), "targets": int(cl[i, 6]), "reads": int(cl[i, 7]),
                "start": round(float(us(cl[i, 0])), 2), "waited": round(float(us(cl[i, 1])), 2),
                "end": round(float(us(cl[i, 2])), 2)} for i in last]
# concurrency: clusters resident at the p50 time
mid = np.percentile(cl[:, 2], 50)
rep["resident_at_p50_end"] = int(((cl[:, 0] <= mid) & (cl[:, 2] >= mid)).sum())
# clusters (and near groups) resident every 50 us
grid = np.arange(0.0, float(us(tr[:, 2]).max()) + 50.0, 50.0)
rep["resident_clusters_50us"] = [int(((us(cl[:, 0]) <= t) & (us(cl[:, 2]) > t)).sum()) for t in grid]
if len(nr):
    rep["resident_near_50us"] = [int(((us(nr[:, 0]) <= t) & (us(nr[:, 2]) > t)).sum()) for t in grid]
xcc = (tr[:, 3] >> 32) & 15
rep["blocks_per_xcc"] = np.bincount(xcc, minlength=8).tolist()
print(json.dumps(rep), flush=True)
