"""The device Arnoldi process (aniso_arnoldi_*, aniso_amd/csrc/arnoldi.hpp: DCGS2 on a
basis that is never rewritten) against plain torch fp64 GMRES (the modified
Gram-Schmidt of gmres.cpp:115-122) on operators whose exact behaviour is known, and
the properties the solver rests on: the orthonormality of Q = P T, the Arnoldi
relation A Q_j = Q_{j+1} H, and bitwise agreement of the one-rank step with its
four-part (sharded) form.  Tolerances: orthonormality and the Arnoldi relation
<= 1e-12; residual histories to 1e-6 relative (rounding-level differences amplified
over a few decades of convergence); solutions <= 1e-10."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


class LowRankOp:
    """A = D + U W^T (n x n, never formed): D diagonal in [1, 1 + spread], U, W n x r random."""

    def __init__(self, n, r, seed, spread=1.0):
        torch = _torch()
        g = torch.Generator(device="cuda").manual_seed(seed)
        self.d = 1.0 + spread * torch.rand(n, dtype=torch.float64, device="cuda", generator=g)
        self.U = (torch.rand(n, r, dtype=torch.float64, device="cuda", generator=g) - 0.5) / np.sqrt(n)
        self.W = (torch.rand(n, r, dtype=torch.float64, device="cuda", generator=g) - 0.5) * 4.0

    def __call__(self, x, y):
        xv = x.reshape(-1)
        y.reshape(-1).copy_(self.d * xv + self.U @ (self.W.t() @ xv))


def _layout(m):
    M1 = m + 1
    Hu = 0
    R = Hu + M1 * m
    T = R + M1 * m
    return {"M1": M1, "Hu": Hu, "R": R, "T": T}


def _mgs_gmres(A, b, m, tol):
    """One cycle of gmres.cpp's MGS Arnoldi in torch fp64: residual estimates per step."""
    torch = _torch()
    nb = float(torch.linalg.norm(b))
    V = [b / nb]
    H = np.zeros((m + 1, m))
    cs, sn, g = np.zeros(m), np.zeros(m), np.zeros(m + 1)
    g[0] = nb
    hist = []
    w = torch.empty_like(b)
    for j in range(m):
        A(V[j], w)
        u = w.clone()
        for i in range(j + 1):
            H[i, j] = float(V[i] @ u)
            u -= H[i, j] * V[i]
        H[j + 1, j] = float(torch.linalg.norm(u))
        V.append(u / H[j + 1, j])
        col = H[:, j].copy()
        for k in range(j):
            t = cs[k] * col[k] + sn[k] * col[k + 1]
            col[k + 1] = -sn[k] * col[k] + cs[k] * col[k + 1]
            col[k] = t
        den = np.hypot(col[j], col[j + 1])
        cs[j], sn[j] = col[j] / den, col[j + 1] / den
        g[j + 1] = -sn[j] * g[j]
        g[j] = cs[j] * g[j]
        hist.append(abs(g[j + 1]) / nb)
        if hist[-1] <= tol:
            break
    return hist


@pytest.mark.parametrize("m", [10, 60, 110])
def test_arnoldi_basis_is_orthonormal_and_satisfies_the_arnoldi_relation(m):
    """m steps of the primitives (m = 60 runs the > 48-row sweeps; m = 110 the small
    kernels past their one-round fast paths: k_arn_coef from j = 64, k_arn_column with
    T staged in LDS up to j = 81 and read from the state block past it, and the
    unstaged k_arn_solve): Q = P T orthonormal and A Q_m = Q_{m+1} H to <= 1e-12,
    residual estimates as torch MGS GMRES, arnoldi_solution = Q_m argmin |beta e_1 - H y|."""
    torch = _torch()
    import aniso_amd
    from aniso_amd import MappedStatus

    a = aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20)  # any handle: the primitives use only its device
    n = 100_003
    A = LowRankOp(n, 70 if m <= 64 else 160, 1)  # rank > m: no convergence to rounding level inside the m steps
    b = torch.rand(n, dtype=torch.float64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    V = torch.zeros(m + 1, n, dtype=torch.float64, device="cuda")
    st = a.arnoldi_state(m)
    stat = MappedStatus()
    V[0].copy_(b)
    nb = float(torch.linalg.norm(b))
    a.arnoldi_begin(V, m, st, nb, status=stat)
    w = torch.empty(n, dtype=torch.float64, device="cuda")
    hist = []
    for j in range(m):
        A(V[j], w)
        a.arnoldi_step(V, m, j, w, st, status=stat)
        torch.cuda.synchronize()
        hist.append(float(stat.host[0]))
        assert int(stat.host[2]) == j + 1
    stat.close()
    ref = _mgs_gmres(A, b, m, 0.0)
    np.testing.assert_allclose(hist, ref, rtol=1e-6, atol=1e-15)
    L = _layout(m)
    M1 = L["M1"]
    T = st[L["T"]:L["T"] + M1 * M1].reshape(M1, M1).t()[:m, :m]  # column-major
    H = st[L["Hu"]:L["Hu"] + M1 * m].reshape(m, M1).t()
    assert float(torch.tril(T, -1).abs().max()) == 0.0
    Q = V[:m].t() @ T  # n x m
    err_o = float((Q.t() @ Q - torch.eye(m, dtype=torch.float64, device="cuda")).abs().max())
    assert err_o <= 1e-12, err_o
    # A Q_{m-1} = Q_m H[:m, :m-1] (the last column's q_m is still raw: compare m - 1 columns)
    AQ = torch.empty_like(Q)
    for k in range(m):
        A(Q[:, k].contiguous(), AQ[:, k])
    lhs = AQ[:, : m - 1]
    rhs = Q @ H[:m, : m - 1]
    err_a = float(torch.linalg.norm(lhs - rhs) / torch.linalg.norm(lhs))
    assert err_a <= 1e-12, err_a
    # the cycle's update x = Q_m y, y the least-squares solution of H y = |b| e_1
    x = torch.zeros(n, dtype=torch.float64, device="cuda")
    a.arnoldi_solution(V, m, m, st, x)
    g = torch.zeros(M1, dtype=torch.float64, device="cuda")
    g[0] = nb
    y = torch.linalg.lstsq(H.cpu(), g.cpu().unsqueeze(1)).solution.squeeze(1).cuda()
    xr = Q @ y
    err_x = float(torch.linalg.norm(x - xr) / torch.linalg.norm(xr))
    assert err_x <= 1e-9, err_x


@pytest.mark.parametrize("restart", [7, 40])
def test_gmres_dist_device_matches_torch_cgs2_and_four_part_form(restart):
    """gmres_dist on the primitives (one rank: aniso_arnoldi_step) against its torch
    CGS2 path: same step counts over restarts, estimates to 1e-6, solutions <= 1e-10;
    and the four-part form (an identity all-reduce between project/coef and
    update/column, the sharded call shape) bitwise equal to the one-rank step."""
    torch = _torch()
    import aniso_amd
    from aniso_amd.solve import gmres_dist

    a = aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20)
    n = 50_001
    A = LowRankOp(n, 12, 5, spread=0.5)
    b = torch.rand(n, dtype=torch.float64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(6))
    h0, h1, h2 = [], [], []
    x0, its0, r0 = gmres_dist(A, b, restart=restart, tol=1e-11, maxit=60, hist=h0)
    x1, its1, r1 = gmres_dist(A, b, restart=restart, tol=1e-11, maxit=60, hist=h1, kry=a)
    x2, its2, r2 = gmres_dist(A, b, restart=restart, tol=1e-11, maxit=60, hist=h2, kry=a,
                              allreduce=lambda t: t)
    assert its0 == its1 == its2 and its1 > 0 and r1 <= 1e-11
    np.testing.assert_allclose(h1, h0, rtol=1e-6, atol=1e-15)
    assert float(torch.linalg.norm(x1 - x0) / torch.linalg.norm(x0)) <= 1e-10
    assert h1 == h2 and torch.equal(x1, x2) and r1 == r2


def test_gmres_dist_device_two_ranks_as_threads():
    """The sharded call shape for real: two ranks as threads, each owning half of the
    rows, their inner products summed by a host all-reduce between the parts; the
    assembled solution equals the one-rank device solve (<= 1e-12) after the same
    number of steps."""
    torch = _torch()
    import aniso_amd
    from aniso_amd.solve import gmres_dist

    n, cut = 40_000, 17_777
    A = LowRankOp(n, 12, 9, spread=0.5)
    b = torch.rand(n, dtype=torch.float64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(10))
    a = aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20)
    xr, itr, rr = gmres_dist(A, b, restart=12, tol=1e-11, maxit=30, kry=a)
    handles = [aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20) for _ in range(2)]
    ranges = [(0, cut), (cut, n)]
    xfull = torch.zeros(n, dtype=torch.float64, device="cuda")
    bar = threading.Barrier(2)
    slots = [None, None]
    res = [None, None]
    errs = []

    def allreduce_for(r):
        def red(t):
            torch.cuda.synchronize()
            slots[r] = t.clone()
            bar.wait()
            tot = slots[0] + slots[1]
            bar.wait()
            t.copy_(tot)
            return t
        return red

    def apply_for(r):
        lo, hi = ranges[r]

        def apply(x, y):
            torch.cuda.synchronize()
            xfull[lo:hi].copy_(x.reshape(-1))
            torch.cuda.synchronize()
            bar.wait()
            yy = torch.empty(n, dtype=torch.float64, device="cuda")
            A(xfull, yy)
            torch.cuda.synchronize()
            bar.wait()
            y.reshape(-1).copy_(yy[lo:hi])
        return apply

    def run(r):
        try:
            lo, hi = ranges[r]
            res[r] = gmres_dist(apply_for(r), b[lo:hi].clone(), restart=12, tol=1e-11, maxit=30,
                                allreduce=allreduce_for(r), kry=handles[r])
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    (x0, it0, r0), (x1, it1, r1) = res
    assert it0 == it1 == itr and r0 == r1 <= 1e-11
    xs = torch.cat([x0, x1])
    assert float(torch.linalg.norm(xs - xr) / torch.linalg.norm(xr)) <= 1e-12
