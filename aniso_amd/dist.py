"""Multi-GPU composition of the sharded apply.

One process per GPU; the targets are sharded by FMM subtree (aniso_set_shard):
each rank owns one contiguous range of the tree order and computes only its
targets.  Per apply (ShardExchange, the multi-GPU GMRES matvec of bench.py):

1. the rank's input is valid at its own range and its halo (aniso_shard_halo: the
   tier-0 subtrees its M2L, near field and correction stencil read);
2. phase 1 (aniso_*_begin_dev) runs the up pass over those subtrees only and packs
   the rank's tier-0 root multipoles; ONE all-gather exchanges them (RCCL over
   xGMI; 2.6 MB at 1M points and 5 right-hand sides);
3. phase 2 (aniso_*_end_dev) scatters them, runs the upper tiers (every rank), the
   M2L and the down pass, writing the owned slice of the next iterate in place;
4. ONE all-to-all sends every rank the halo of the next iterate from its owners.

The older replicated scheme (whole input on every rank, full up pass, all-gather of
the output slices: gather_index / block_gather_index / assemble_from_gathered) is
kept for the original-order and single-phase tests.
"""
import numpy as np


def _is_torch(x):
    try:
        import torch
    except ImportError:
        return False
    return isinstance(x, torch.Tensor)


def shard_ranges(op, nranks):
    """[(begin, end)] tree-order ranges of every shard, computed host-side without
    changing the handle's shard or caches (aniso_shard_cuts)."""
    c = op.shard_cuts(nranks)
    return [(int(c[r]), int(c[r + 1])) for r in range(nranks)]


def pad_len(ranges):
    return max(e - b for b, e in ranges) if ranges else 0


def assemble_from_gathered(gathered, ranges, perm, out=None):
    """gathered: (nranks, L) tree-ordered slices (numpy or torch); returns the
    original-order vector out[perm[k]] = tree[k]."""
    if _is_torch(gathered):
        import torch

        parts = [gathered[r, : e - b] for r, (b, e) in enumerate(ranges)]
        tree = torch.cat(parts)
        if out is None:
            out = torch.empty_like(tree)
        out[perm] = tree
        return out
    tree = np.concatenate([gathered[r, : e - b] for r, (b, e) in enumerate(ranges)])
    if out is None:
        out = np.empty_like(tree)
    out[perm] = tree
    return out


def local_slice(full_orig, perm, rng, L):
    """Tree-order slice of this rank's owned targets, padded to length L."""
    b, e = rng
    if _is_torch(full_orig):
        import torch

        buf = torch.zeros(L, dtype=full_orig.dtype, device=full_orig.device)
        buf[: e - b] = full_orig[perm[b:e]]
        return buf
    buf = np.zeros(L, dtype=full_orig.dtype)
    buf[: e - b] = full_orig[perm[b:e]]
    return buf


def gather_index(ranges, L):
    """Positions in the flattened (nranks, L) all-gather buffer of tree positions
    0 .. N-1: tree[k] = gathered.reshape(-1)[idx[k]]."""
    return np.concatenate([r * L + np.arange(e - b, dtype=np.int64) for r, (b, e) in enumerate(ranges)])


def block_gather_index(ranges, L, nb):
    """Positions in the flattened (nranks, nb, L) all-gather buffer of the block
    vector (nb, N) in tree order: y.reshape(-1)[b * N + k] = gathered.reshape(-1)[idx]."""
    g = gather_index(ranges, L)
    r, off = g // L, g % L
    return np.concatenate([r * nb * L + b * L + off for b in range(nb)])


def _intersect(ranges, b, e):
    """Positions of the [b_i, e_i) pairs that fall inside [b, e), ascending."""
    parts = [np.arange(max(lo, b), min(hi, e), dtype=np.int64) for lo, hi in ranges if min(hi, e) > max(lo, b)]
    return np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)


def halo_plan(cuts, halos, rank):
    """Host-side halo exchange of one rank: (send[r], recv[r]) tree positions it sends
    to / receives from rank r.  cuts: nranks + 1 shard boundaries; halos[r]: rank r's
    aniso_shard_halo ranges.  A rank sends to r the positions of r's halo inside its
    own range; it receives from r the positions of its halo inside r's range."""
    n = len(cuts) - 1
    b, e = int(cuts[rank]), int(cuts[rank + 1])
    send = [_intersect(halos[r], b, e) if r != rank else np.zeros(0, dtype=np.int64) for r in range(n)]
    recv = [_intersect(halos[rank], int(cuts[r]), int(cuts[r + 1])) if r != rank else np.zeros(0, dtype=np.int64)
            for r in range(n)]
    return send, recv


class ShardExchange:
    """The two collectives of one rank's sharded apply (module docstring): the root
    all-gather between aniso_*_begin_dev and aniso_*_end_dev, and the halo
    all-to-all of the next iterate.  nb vectors (blocks) of N points in tree order
    per iterate; backend "nccl" (RCCL, device buffers) or "gloo" (staged through
    host memory: CPU tests and one-GPU rehearsals)."""

    def __init__(self, op, rank, world, nb, device, backend="nccl"):
        import torch
        import torch.distributed as dist

        self.dist, self.torch = dist, torch
        self.rank, self.world, self.nb, self.N = rank, world, nb, op.N
        self.backend = backend
        ex = op.shard_exchange(nb)
        self.C, self.R = ex["root_chunk"], ex["root_record"]
        n = max(self.C * self.R, 1)
        self.roots_send = torch.zeros(n, dtype=torch.float64, device=device)
        self.roots_recv = torch.zeros(world * n, dtype=torch.float64, device=device)
        self.cuts = op.shard_cuts(world)
        self.own = (int(self.cuts[rank]), int(self.cuts[rank + 1]))
        mine = [tuple(int(v) for v in r) for r in op.shard_halo()]
        halos = [None] * world
        dist.all_gather_object(halos, mine)  # setup only (host)
        self.halos = halos
        send, recv = halo_plan(self.cuts, halos, rank)
        self.send_pos, self.recv_pos = send, recv
        blk = np.arange(nb, dtype=np.int64)[:, None] * self.N
        cat = lambda pos: np.concatenate([(blk + p[None, :]).reshape(-1) for p in pos])  # noqa: E731 [peer][b][pos]
        self.in_splits = [nb * len(p) for p in send]
        self.out_splits = [nb * len(p) for p in recv]
        self.send_idx = torch.tensor(cat(send), device=device)
        self.recv_idx = torch.tensor(cat(recv), device=device)
        self.send_buf = torch.zeros(max(sum(self.in_splits), 1), dtype=torch.float64, device=device)
        self.recv_buf = torch.zeros(max(sum(self.out_splits), 1), dtype=torch.float64, device=device)

    def roots_allgather(self):
        if self.C == 0:
            return
        if self.backend == "nccl":
            self.dist.all_gather_into_tensor(self.roots_recv, self.roots_send)
            return
        parts = [self.torch.zeros_like(self.roots_send, device="cpu") for _ in range(self.world)]
        self.dist.all_gather(parts, self.roots_send.cpu())
        self.roots_recv.copy_(self.torch.cat(parts))

    def halo(self, y):
        """Fill y's halo (y: (nb, N) tree order, own slice already written) from its owners."""
        flat = y.view(-1)
        ns, nr = sum(self.in_splits), sum(self.out_splits)
        if ns:
            self.torch.index_select(flat, 0, self.send_idx, out=self.send_buf[:ns])
        if self.backend == "nccl":
            self.dist.all_to_all_single(self.recv_buf[:nr], self.send_buf[:ns], self.out_splits, self.in_splits)
            if nr:
                flat.index_copy_(0, self.recv_idx, self.recv_buf[:nr])
            return
        rb = self.torch.zeros(nr, dtype=self.torch.float64)
        self.dist.all_to_all_single(rb, self.send_buf[:ns].cpu(), self.out_splits, self.in_splits)
        if nr:
            flat.index_copy_(0, self.recv_idx, rb.to(y.device))

    def halo_bytes(self):
        return 8 * sum(self.out_splits)
