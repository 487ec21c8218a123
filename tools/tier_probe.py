"""Per-phase timing of the up/down tier kernels from the probe build (make -C
aniso_amd/csrc probe): ANISO_LIB=aniso_amd/libaniso_probe.so python tools/tier_probe.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import gaussian, main_coeffs  # noqa: E402

block = "--block" in sys.argv  # the aniso.m block matvec (K = 5) instead of mode 0
op = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
ss, st = main_coeffs(xy)
op.setCoeff(ss, st)
perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
if block:
    for m in range(9):
        op.cache(m)
    x = torch.zeros(5, op.N, dtype=torch.float64, device="cuda")
    x[0] = torch.tensor(gaussian(xy), device="cuda")[perm]
    y = torch.zeros_like(x)
    for _ in range(5):
        op.block_op_dev(2, x, y, tree=True)
else:
    op.cache(0)
    x = torch.tensor(gaussian(xy), device="cuda")[perm].contiguous()
    y = torch.zeros_like(x)
    for _ in range(5):
        op.forward_tree_dev(x, y)
torch.cuda.synchronize()
L = aniso_amd.lib()
buf = np.zeros((2, 8192, 8), dtype=np.uint64)
fn = L.aniso_probe_read
fn.argtypes = [ctypes.c_void_p]
fn.restype = ctypes.c_int
assert fn(buf.ctypes.data) == 0
# tier task ranges of the uniform 1M tree (D = 8): bottom tier roots at D - bspan + 1,
# upper tiers every tspan levels up to level 1 (host_tree.cpp Plan::build)
D = 8
bspan = int(os.environ.get("ANISO_BOTTOM_SPAN", "3"))
tspan = int(os.environ.get("ANISO_TOP_SPAN", "2"))
roots = [max(1, D - bspan + 1)]
while roots[-1] > 1:
    roots.append(max(1, roots[-1] - tspan))
sels, t0_ = [], 0
for i, r in enumerate(roots):
    sels.append((0, f"up tier {i} (root level {r})", slice(t0_, t0_ + 4 ** r)))
    t0_ += 4 ** r
sels.append((1, "down (all tasks)", slice(0, 8192)))
for k, name, sel in sels:
    nph = 5
    b = buf[k][sel].astype(np.int64)
    used = b[:, 0] > 0
    b = b[used]
    t0 = b[:, 0].min()
    print(name, "workgroups", used.sum(), "span us", (b[:, nph - 1].max() - t0) / 100.0)
    for i in range(1, nph):
        d = (b[:, i] - b[:, i - 1]) / 100.0  # wall_clock64 at 100 MHz
        print(f"  phase {i}: mean {d.mean():7.2f} us  max {d.max():7.2f} us")
    st_ = (b[:, 0] - t0) / 100.0
    wg = np.nonzero(used)[0]
    per_x = [np.median(st_[(wg % 8) == x]) for x in range(8)] if len(wg) >= 8 else []
    print("  median start by blockIdx % 8:", " ".join(f"{v:.2f}" for v in per_x))
    print(f"  start skew: max {st_.max():.2f} us; percentiles 25/50/75/90: "
          f"{np.percentile(st_, 25):.2f} {np.percentile(st_, 50):.2f} {np.percentile(st_, 75):.2f} {np.percentile(st_, 90):.2f}")
