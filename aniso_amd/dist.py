"""Multi-GPU composition of the sharded apply.

One process per GPU.  Every rank holds the whole input vector (GMRES vectors are
replicated), runs the cheap up pass redundantly, and computes the targets of its
FMM-subtree shard only (aniso_set_shard): those targets form one contiguous range
of the tree order.  The output is assembled with ONE all-gather of the tree-ordered
shard slices (RCCL over xGMI on the GPU box, gloo on CPU).  With the vectors kept
in tree order (aniso_forward_tree_dev) the assembly is a single index gather of
the padded all-gather buffer (gather_index); with original-order vectors it is a
permutation (assemble_from_gathered).  No other collective is on the data path.
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
