"""Per-rank block-matvec time of one shard: what one GPU of an N-GPU strong-scaling
run computes per step, in the two phases of the sharded apply with
the root all-gather replaced by a device copy of this rank's own contribution
(the collectives are not timed here).  usage: shard_time.py WORLD [RANK...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
timing = "--no-timing" not in sys.argv  # --no-timing: no stage events (they add packets between the kernels)
native = "--native" in sys.argv  # the library's one-call sharded matvec over a loopback communicator
world = int(args[0]) if args else 8
ranks = [int(a) for a in args[1:]] or [0]
for rank in ranks:
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
    if native and world > 1:
        op.comm_init_loopback()
    send = torch.zeros(max(C * R, 1), dtype=torch.float64, device="cuda")
    recv = torch.zeros(world * max(C * R, 1), dtype=torch.float64, device="cuda")

    def step():
        if world == 1:
            op.block_op_dev(2, x, y, tree=True)
            return
        if native:
            op.block_op_sharded_dev(2, x, y)
            return
        op.block_op_begin_dev(2, x, y[:, b:e], send)
        recv[rank * C * R:(rank + 1) * C * R].copy_(send[: C * R])  # stands in for the all-gather
        op.block_op_end_dev(2, x, y[:, b:e], recv, world)

    for _ in range(3):
        step()
    op.set_timing(timing)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps = 20
    for _ in range(steps):
        step()
    host_ms = 1e3 * (time.perf_counter() - t0) / steps  # enqueue time: close to ms = host-bound
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    st = op.stats()
    print(json.dumps({"world": world, "rank": rank, "native": native, "ms_per_apply": round(ms, 4), "host_ms_per_apply": round(host_ms, 4),
                      "stage_ms": {k: round(v, 4) for k, v in op.stage_times().items()} if timing else None,
                      "t0_tasks_run": ex["t0_run"], "t0_tasks": ex["t0_tasks"], "halo_points": ex["halo_points"],
                      "m2l_clusters": st["hm_clusters"], "m2l_targets": st["m2l_targets"], "leaves": st["leaves"]}),
          flush=True)
    del op
