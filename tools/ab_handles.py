"""Same-process A/B of environment knobs on the 1M-point block matvec (or one rank of
an N-way shard): one handle per configuration (knobs are read at handle creation),
timed in interleaved repetitions so box drift hits every configuration alike.
usage: ab_handles.py [--world W] [--rank R] [--steps S] [--reps P] CFG [CFG ...]
CFG = "" (defaults) or "ANISO_X=a,ANISO_Y=b"."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian, main_coeffs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--sz", type=int, default=1024)
ap.add_argument("--ks", type=int, default=5, help="5: aniso.m block matvec; 1: main.cpp forward operator (mode 0)")
ap.add_argument("cfgs", nargs="+")
args = ap.parse_args()
world, rank = args.world, args.rank
runs = []
for cfg in args.cfgs:
    kv = [c.split("=", 1) for c in cfg.split(",") if c]
    saved = {k: os.environ.get(k) for k, _ in kv}
    for k, v in kv:
        os.environ[k] = v
    op = aniso_amd.Aniso(args.sz, 1, args.ks, 0.8, 10, 4, 20)
    if world > 1:  # the shard's plan is built here: under the same knobs
        op.set_shard(rank, world)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    xy = op.getNodes()
    perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
    op.setCoeff(*(demo_coeffs(xy) if args.ks > 1 else main_coeffs(xy)))
    for m in range(2 * args.ks - 1):
        op.cache(m)
    b, e = op.shard()
    ex = op.shard_exchange(args.ks)
    C, R = ex["root_chunk"], ex["root_record"]
    x = torch.zeros(args.ks, op.N, dtype=torch.float64, device="cuda")
    x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
    y = torch.zeros_like(x)
    send = torch.zeros(max(C * R, 1), dtype=torch.float64, device="cuda")
    recv = torch.zeros(world * max(C * R, 1), dtype=torch.float64, device="cuda")
    runs.append(dict(cfg=cfg or "default", op=op, x=x, y=y, send=send, recv=recv, b=b, e=e, C=C, R=R, ms=[], st=None))


def step(r):
    op, x, y = r["op"], r["x"], r["y"]
    b, e, C, R = r["b"], r["e"], r["C"], r["R"]
    if world == 1:
        if args.ks > 1:
            op.block_op_dev(2, x, y, tree=True)
        else:
            op.forward_tree_dev(x[0], y[0])
        return
    if args.ks > 1:
        op.block_op_begin_dev(2, x, y[:, b:e], r["send"])
    else:
        op.forward_tree_begin_dev(x[0], y[0, b:e], r["send"])
    r["recv"][rank * C * R:(rank + 1) * C * R].copy_(r["send"][: C * R])  # stands in for the all-gather
    if args.ks > 1:
        op.block_op_end_dev(2, x, y[:, b:e], r["recv"], world)
    else:
        op.forward_tree_end_dev(x[0], y[0, b:e], r["recv"], world)


for rep in range(args.reps):
    for r in runs:
        for _ in range(3):
            step(r)
        r["op"].set_timing(rep == args.reps - 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(r)
        torch.cuda.synchronize()
        r["ms"].append(round(1e3 * (time.perf_counter() - t0) / args.steps, 4))
        if rep == args.reps - 1:
            r["st"] = {k: round(v, 4) for k, v in r["op"].stage_times().items()}
            r["op"].set_timing(False)
        r["op"].sync()
ref = runs[0]["y"][:, runs[0]["b"]:runs[0]["e"]]
for r in runs:
    s = r["op"].stats()
    d = r["y"][:, r["b"]:r["e"]]
    rel = float(torch.linalg.norm(d - ref) / torch.linalg.norm(ref))  # same input: outputs agree to rounding
    print(json.dumps({"cfg": r["cfg"], "world": world, "rank": rank, "ms": r["ms"], "best_ms": min(r["ms"]),
                      "stage_ms": r["st"], "clusters": s["hm_clusters"],
                      "block_reads": s["hm_block_reads"], "dual_pairs": s["hm_dual_pairs"],
                      "rel_vs_first": rel}), flush=True)
