"""The library's one-call sharded matvec (aniso_block_op_sharded_dev: halo all-to-all,
phase 1, RCCL root all-gather, phase 2) against the Python-orchestrated one
(aniso_amd.dist.ShardExchange between aniso_block_op_begin_dev / _end_dev), on a
one-rank shard of the 1M-point problem with a real RCCL communicator: what the host
round trips between the phases cost.  usage (one GPU):
python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/comm_ab.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import aniso_amd  # noqa: E402
from aniso_amd import dist as adist  # noqa: E402
from bench import demo_coeffs, gaussian  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = 30
op = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
op.set_shard(0, 1)
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
xchg = adist.ShardExchange(op, 0, 1, 5, "cuda", "nccl")
adist.native_comm_init(op, 1, "nccl")
ob, oe = xchg.own
x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
y = torch.zeros_like(x)


def py_step(a, b):
    op.block_op_begin_dev(2, a, b[:, ob:oe], xchg.roots_send)
    xchg.roots_allgather()
    op.block_op_end_dev(2, a, b[:, ob:oe], xchg.roots_recv, 1)
    xchg.halo(b)


def native_step(a, b):
    op.block_op_sharded_dev(2, a, b)


res = {"N": op.N}
for rep in range(3):
    for name, fn in (("python", py_step), ("native", native_step)):
        for _ in range(3):
            fn(x, y)
            x, y = y, x
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn(x, y)
            x, y = y, x
        host = 1e3 * (time.perf_counter() - t0) / steps
        torch.cuda.synchronize()
        res.setdefault(f"{name}_ms", []).append(round(1e3 * (time.perf_counter() - t0) / steps, 4))
        res.setdefault(f"{name}_host_enqueue_ms", []).append(round(host, 4))
# the RCCL all-gather alone (the tier-0 root records: 4,096 x 16 x 5 doubles at 1M points)
buf = torch.rand(xchg.C * xchg.R, dtype=torch.float64, device="cuda")
out = torch.zeros_like(buf)
for _ in range(5):
    dist.all_gather_into_tensor(out, buf)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    dist.all_gather_into_tensor(out, buf)
torch.cuda.synchronize()
res["rccl_allgather_one_rank_us"] = round(1e6 * (time.perf_counter() - t0) / 100, 2)
res["root_record_bytes"] = 8 * xchg.C * xchg.R
dist.destroy_process_group()
print(json.dumps(res), flush=True)
