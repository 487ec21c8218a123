"""The N>1 path's composition on CPU with gloo (world_size 2 and 3): every rank
owns an FMM-subtree shard (a contiguous tree-order range), computes its targets,
and one all-gather of the tree-ordered slices + a permutation rebuilds the full
vector.  The per-rank compute is played by the oracle here (no GPU on CPU); on
the GPU box the same composition runs over RCCL with the HIP apply (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import aniso_amd
    from aniso_amd import dist as adist
    from oracle.oracle_py import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sz, d = 12, 2
        a = aniso_amd.Aniso(sz, d, 2, 0.5, 8, 4, 20)
        ranges = adist.shard_ranges(a, world)
        a.set_shard(rank, world)
        assert a.shard() == ranges[rank]
        perm = a.tree_perm()
        o = Oracle(sz, d, 2, 0.5, 8, 4, 20)
        xy = o.getNodes()
        rng = np.random.default_rng(7)
        o.setCoeff(rng.uniform(1, 2, o.N), rng.uniform(2, 3, o.N))
        o.cache(1)
        q = rng.uniform(-1, 1, o.N)
        full = o.mapping(q, 1)  # every rank can compute it: stands in for the shard's apply
        L = adist.pad_len(ranges)
        mine = torch.from_numpy(adist.local_slice(full, perm, ranges[rank], L))
        parts = [torch.zeros(L, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, mine)
        gathered = torch.stack(parts)
        out = adist.assemble_from_gathered(gathered.numpy(), ranges, perm)
        result_q.put((rank, float(np.abs(out - full).max()), xy.shape[0]))
    except Exception as e:  # surface worker failures instead of hanging the queue
        result_q.put((rank, repr(e), -1))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_assembly(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, err, n in res:
        assert n > 0, err
        assert err == 0.0, (r, err)


def test_block_gather_index_assembles_block_slices():
    from aniso_amd import dist as adist

    ranges = [(0, 5), (5, 7), (7, 13)]
    L, nb, N = 6, 3, 13
    full = np.arange(nb * N, dtype=np.float64).reshape(nb, N)
    gathered = np.zeros((3, nb, L))
    for r, (b, e) in enumerate(ranges):
        gathered[r, :, : e - b] = full[:, b:e]
    idx = adist.block_gather_index(ranges, L, nb)
    assert np.array_equal(gathered.reshape(-1)[idx].reshape(nb, N), full)
