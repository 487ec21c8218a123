#!/usr/bin/env python3
"""Fraction of V-list pairs (uniform quadtree level L) whose both ends fall in the same
2^k x 2^k cluster of same-level nodes: the pairs a cluster workgroup can apply from
one read of a stored block."""
import sys


def vlist(L):
    n = 2 ** L
    V = {}
    for x in range(n):
        for y in range(n):
            px, py = x // 2, y // 2
            V[(x, y)] = [(cx, cy) for cx in range(2 * px - 2, 2 * px + 4) for cy in range(2 * py - 2, 2 * py + 4)
                         if 0 <= cx < n and 0 <= cy < n and max(abs(cx - x), abs(cy - y)) >= 2]
    return V


L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
V = vlist(L)
D = sum(len(v) for v in V.values())
for k in range(1, min(L, 6) + 1):
    inner = sum(1 for a, v in V.items() for b in v if a[0] >> k == b[0] >> k and a[1] >> k == b[1] >> k)
    f = inner / D
    print(f"k={k} cluster={4 ** k:5d} internal={f:.3f} blocks read / directed={1 - f / 2:.3f}")
