"""RCCL check of the sharded apply's two collectives (aniso_amd/dist.py ShardExchange)
on a one-GPU box: one rank, backend "nccl" (= RCCL on ROCm), the same calls, dtypes and
buffer shapes bench.py issues at N > 1 (all_gather_into_tensor of the tier-0 root
records, all_to_all_single of the halo, with and without an empty exchange).
RCCL refuses two ranks on one device, so one rank sending to itself is what a one-GPU
box can check; the multi-rank plans are covered by tests/test_dist_cpu.py (gloo).
usage: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/rccl_check.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from aniso_amd.dist import ShardExchange  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    assert dist.get_backend() == "nccl"
    nb, N = 5, 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    res = {}

    ex = ShardExchange.__new__(ShardExchange)  # the collectives only; plans come from tests/test_dist_cpu.py
    ex.dist, ex.torch, ex.backend, ex.world, ex.rank, ex.nb, ex.N = dist, torch, "nccl", 1, 0, nb, N
    # root all-gather: 4,096 records of 16 x 5 doubles (1M points), as at N ranks
    ex.C, ex.R = 4096, 16 * nb
    ex.roots_send = torch.rand(ex.C * ex.R, dtype=torch.float64, device="cuda", generator=g)
    ex.roots_recv = torch.zeros_like(ex.roots_send)
    ex.roots_allgather()
    torch.cuda.synchronize()
    res["allgather_equal"] = bool(torch.equal(ex.roots_recv, ex.roots_send))

    # halo all-to-all: positions [0, 300) of every block refresh [N-300, N) (self-send)
    pos = torch.arange(300, device="cuda")
    blk = torch.arange(nb, device="cuda")[:, None] * N
    ex.send_idx = (blk + pos[None, :]).reshape(-1)
    ex.recv_idx = (blk + (N - 300 + pos)[None, :]).reshape(-1)
    ex.in_splits, ex.out_splits = [nb * 300], [nb * 300]
    ex.send_buf = torch.zeros(nb * 300, dtype=torch.float64, device="cuda")
    ex.recv_buf = torch.zeros_like(ex.send_buf)
    y = torch.rand(nb, N, dtype=torch.float64, device="cuda", generator=g)
    want = y.clone()
    want[:, N - 300:] = y[:, :300]
    ex.halo(y)
    torch.cuda.synchronize()
    res["halo_equal"] = bool(torch.equal(y, want))
    res["halo_bytes"] = ex.halo_bytes()

    # a rank with no halo: empty splits through RCCL leave y untouched
    ex.in_splits, ex.out_splits = [0], [0]
    before = y.clone()
    ex.halo(y)
    torch.cuda.synchronize()
    res["empty_halo_untouched"] = bool(torch.equal(y, before))
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(res))
    ok = res["allgather_equal"] and res["halo_equal"] and res["empty_halo_untouched"]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
