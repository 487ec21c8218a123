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

GMRES over the shards (aniso_amd.solve.gmres_dist) adds two all-reduces of its
inner products per Arnoldi step (ShardExchange.allreduce).
"""
import numpy as np


def shard_ranges(op, nranks):
    """[(begin, end)] tree-order ranges of every shard, computed host-side without
    changing the handle's shard or caches (aniso_shard_cuts)."""
    c = op.shard_cuts(nranks)
    return [(int(c[r]), int(c[r + 1])) for r in range(nranks)]


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

    def allreduce(self, t):
        """Sum a small float64 tensor over the ranks in place (GMRES inner products,
        aniso_amd.solve.gmres_dist: two per Arnoldi step)."""
        if self.backend == "nccl":
            self.dist.all_reduce(t)
            return t
        c = t.cpu()
        self.dist.all_reduce(c)
        t.copy_(c)
        return t


def sharded_block_matvec(op, xchg, which=2):
    """apply(x, y) for aniso_amd.solve.gmres_dist on one rank's owned slices: x, y
    are (nb, n_own) tree-order slices of the iterate.  The slice is placed into a
    full-length work vector whose halo the all-to-all then fills from its owners;
    phase 1, the root all-gather and phase 2 write y (x - mforward(x) for which = 2)."""
    import torch

    ob, oe = xchg.own
    full = torch.zeros(xchg.nb, op.N, dtype=torch.float64, device=xchg.roots_send.device)

    def apply(x, y):
        full[:, ob:oe] = x
        xchg.halo(full)
        op.block_op_begin_dev(which, full, y, xchg.roots_send)
        xchg.roots_allgather()
        op.block_op_end_dev(which, full, y, xchg.roots_recv, xchg.world)

    return apply


class HostCollectives:
    """aniso_collectives over a torch.distributed group with host staging (gloo): the
    library's own exchange (aniso_comm_init_callbacks) driven through CPU collectives,
    so several ranks may share one GPU (RCCL refuses that).  copy(dst, src, nbytes)
    moves bytes between device and host addresses (aniso_amd.memcpy; tests on the
    CPU pass ctypes.memmove)."""

    def __init__(self, world, copy=None):
        import ctypes

        import torch.distributed as dist

        import aniso_amd

        self.world, self.dist = world, dist
        self.copy = copy or aniso_amd.memcpy
        self.errors = []
        self.struct = aniso_amd.Collectives(None, aniso_amd.COLL_ALLGATHER(self._allgather),
                                            aniso_amd.COLL_ALLTOALLV(self._alltoallv),
                                            aniso_amd.COLL_ALLREDUCE(self._allreduce))
        self._ct = ctypes

    def _host(self, ptr, n):
        buf = np.empty(int(n), dtype=np.float64)
        if n:
            self.copy(buf.ctypes.data, ptr, 8 * int(n))
        return buf

    def _back(self, ptr, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if arr.size:
            self.copy(ptr, arr.ctypes.data, 8 * arr.size)

    def _guard(self, fn):
        try:
            fn()
            return 0
        except Exception as ex:  # a failure becomes the callback's status (the library raises)
            self.errors.append(repr(ex))
            return 1

    def _allgather(self, ctx, send, recv, count, stream):
        import torch

        def run():
            t = torch.from_numpy(self._host(send, count))
            parts = [torch.empty(int(count), dtype=torch.float64) for _ in range(self.world)]
            self.dist.all_gather(parts, t)
            self._back(recv, torch.cat(parts).numpy())
        return self._guard(run)

    def _alltoallv(self, ctx, send, scount, soff, recv, rcount, roff, stream):
        import torch

        def run():
            sc = [int(scount[p]) for p in range(self.world)]
            rc = [int(rcount[p]) for p in range(self.world)]
            so = [int(soff[p]) for p in range(self.world)]
            ro = [int(roff[p]) for p in range(self.world)]
            sbuf = self._host(send, max((o + c for o, c in zip(so, sc)), default=0))
            st = torch.from_numpy(np.concatenate([sbuf[o:o + c] for o, c in zip(so, sc)]) if sum(sc) else np.zeros(0))
            rt = torch.empty(sum(rc), dtype=torch.float64)
            self.dist.all_to_all_single(rt, st, rc, sc)
            r = rt.numpy()
            pos = 0
            for o, c in zip(ro, rc):
                if c:
                    self._back(recv + 8 * o, r[pos:pos + c])
                pos += c
        return self._guard(run)

    def _allreduce(self, ctx, buf, count, stream):
        import torch

        def run():
            t = torch.from_numpy(self._host(buf, count))
            self.dist.all_reduce(t)
            self._back(buf, t.numpy())
        return self._guard(run)


def native_comm_init(op, world, backend="nccl"):
    """Attach the library's own communicator to a sharded handle (every rank together):
    RCCL from a unique id broadcast over torch.distributed, or the host-staged
    callbacks (gloo).  Returns the callbacks object (keep it alive) or None."""
    import torch.distributed as dist

    import aniso_amd

    if backend == "nccl":
        uid = [aniso_amd.comm_unique_id() if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        op.comm_init_rccl(uid[0])
        return None
    coll = HostCollectives(world)
    op.comm_init_callbacks(coll.struct)
    return coll


def native_block_matvec(op, nb, device, which=2):
    """apply(x, y) for aniso_amd.solve.gmres_dist on this rank's owned slices over the
    library's one-call sharded operator (aniso_block_op_sharded_dev)."""
    import torch

    b, e = op.shard()
    fx = torch.zeros(nb, op.N, dtype=torch.float64, device=device)
    fy = torch.zeros_like(fx)

    def apply(x, y):
        fx[:, b:e] = x
        op.block_op_sharded_dev(which, fx, fy)
        y.copy_(fy[:, b:e])

    return apply
