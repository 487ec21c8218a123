"""Element-level check of aniso_krylov_update against torch (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, aniso_amd
a = aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20)
for nv in (16, 17, 24, 32, 33, 40):
    for n in (300007, 2048 * 256, 1000):
        g = torch.Generator(device="cuda").manual_seed(nv)
        V = torch.rand(nv, n, dtype=torch.float64, device="cuda", generator=g) - 0.5
        w = torch.rand(n, dtype=torch.float64, device="cuda", generator=g) - 0.5
        c = torch.rand(nv, dtype=torch.float64, device="cuda", generator=g) - 0.5
        out = torch.zeros(nv + 1, dtype=torch.float64, device="cuda")
        w1 = w.clone()
        a.krylov_update(V, c, w1, out, dots=True)
        wr = w - V.t() @ c
        bad = ((w1 - wr).abs() > 1e-10).nonzero().flatten()
        w2 = w.clone(); sq = torch.zeros(1, dtype=torch.float64, device="cuda")
        a.krylov_update(V, c, w2, sq, dots=False)
        bad2 = ((w2 - wr).abs() > 1e-10).nonzero().flatten()
        print(nv, n, "bad dots-mode:", bad.numel(), bad[:5].tolist(), bad[-3:].tolist(), "bad norm-mode:", bad2.numel(), flush=True)
