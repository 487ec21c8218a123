"""Multi-right-hand-side, mixed-precision GMRES over the device block apply
(the a15 caller, main.cpp:121-141 / gmres.cpp:53-169,
for k right-hand sides at once).

    A(u) = u - K_0(sigma_s .* u)     (main.cpp:125-136 forwardOperator, mode 0)

* The operator runs in fp64 on the MI355X: `Aniso.apply_block_dev` applies K_0 to
  up to 8 right-hand sides per launch sequence from one read of the cached
  operators; 16 right-hand sides are two batches.
* Inner solver: restarted GMRES(m) with the Krylov basis stored in fp32 (modified
  Gram-Schmidt; dot products accumulated in fp64), Givens rotations per right-hand
  side on the host, to a loose relative tolerance.
* Outer loop: iterative refinement in fp64, r = b - A x, x += inner(r), until
  ||r|| / ||b|| <= tol for every right-hand side.

* Inner operator for 16 right-hand sides: the fp32 MFMA operator
  (`Aniso.forward_f32_dev`: fp32 caches, every FMM translation a 16 x 16 x 16
  v_mfma_f32_16x16x4_f32 product) on tree-order, point-major
  vectors.  The outer residuals use the fp64 operator.

This is host orchestration over torch tensors (device memory and BLAS-1 plumbing);
the operators it calls are the HIP path.
"""
import numpy as np

MAX_BATCH = 8


class MT19937_64:
    """std::mt19937_64 (the survey's config-5 centre generator)."""

    def __init__(self, seed):
        self.mt = [0] * 312
        self.mt[0] = seed & 0xFFFFFFFFFFFFFFFF
        for i in range(1, 312):
            p = self.mt[i - 1]
            self.mt[i] = (6364136223846793005 * (p ^ (p >> 62)) + i) & 0xFFFFFFFFFFFFFFFF
        self.i = 312

    def _twist(self):
        mt = self.mt
        for i in range(312):
            x = (mt[i] & 0xFFFFFFFF80000000) | (mt[(i + 1) % 312] & 0x7FFFFFFF)
            xa = x >> 1
            if x & 1:
                xa ^= 0xB5026F5AA96619E9
            mt[i] = mt[(i + 156) % 312] ^ xa
        self.i = 0

    def __call__(self):
        if self.i >= 312:
            self._twist()
        y = self.mt[self.i]
        self.i += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & 0xFFFFFFFFFFFFFFFF

    def uniform(self, a, b):
        """std::uniform_real_distribution<double>(a, b) as libstdc++ draws it from a
        64-bit engine: one draw, generate_canonical = double(g()) / 2^64."""
        r = float(self()) / 18446744073709551616.0
        if r >= 1.0:
            r = np.nextafter(1.0, 0.0)
        return a + (b - a) * r


def config5_charges(xy, k, width=25.0):
    """q_k = exp(-width |x - c_k|^2), c_k uniform in [0.2, 0.8]^2 from mt19937_64(seed=k)."""
    g = MT19937_64(k)
    cx = g.uniform(0.2, 0.8)
    cy = g.uniform(0.2, 0.8)
    return np.exp(-width * ((xy[:, 0] - cx) ** 2 + (xy[:, 1] - cy) ** 2))


def forward_block(op, X, Y):
    """Y = X - K_0(sigma_s .* X) for the rows of X (fp64 device tensors), <= 8 per apply."""
    for b0 in range(0, X.shape[0], MAX_BATCH):
        xs, ys = X[b0:b0 + MAX_BATCH], Y[b0:b0 + MAX_BATCH]
        k = xs.shape[0]
        op.apply_block_dev(xs, [0], np.eye(k)[None], ys, use_sigma=True)
        ys.neg_().add_(xs)


def forward16(op, X, W, perm):
    """W = X - K_0(sigma_s .* X) for 16 rows on the fp64 MFMA operator
    (Aniso.forward16_f64_dev: tree order, point-major; every FMM translation a
    16 x 16 x 16 v_mfma_f64_16x16x4_f64 product)."""
    import torch

    X16 = X[:, perm].t().contiguous()
    Y16 = torch.empty_like(X16)
    op.forward16_f64_dev(X16, Y16)
    W[:, perm] = Y16.t()


def rhs_block(op, Q):
    """rhs_k = K_0 q_k (main.cpp:121-124: the right-hand side is the mapping of q)."""
    import torch

    R = torch.empty_like(Q)
    for b0 in range(0, Q.shape[0], MAX_BATCH):
        qs = Q[b0:b0 + MAX_BATCH]
        op.apply_block_dev(qs, [0], np.eye(qs.shape[0])[None], R[b0:b0 + MAX_BATCH], use_sigma=False)
    return R


def _inner_gmres(apply, R, m, tol, max_cycles, rd=1):
    """Approximately solve A D = R (right-hand sides independent) with an fp32 Krylov
    basis.  rd: the axis of R that runs over the points (1: R is (k, n), the fp64
    operator's row layout; 0: (n, k), the fp32 operator's point-major layout).
    apply(X, W): W = A X in R's layout (X may be fp32 or fp64, W fp64)."""
    import torch

    k = R.shape[1 - rd]

    def col(v):  # per-right-hand-side scalars broadcast along the points
        return v[:, None] if rd == 1 else v[None, :]

    D = torch.zeros_like(R)
    r0 = torch.linalg.norm(R, dim=rd).cpu().numpy()
    W = torch.empty_like(R)
    its = 0
    for _ in range(max_cycles):
        Rc = R.clone()
        if its:
            apply(D, W)
            Rc -= W
        beta = torch.linalg.norm(Rc, dim=rd).cpu().numpy()
        done = beta <= tol * r0
        if done.all():
            break
        V = torch.zeros((m + 1,) + tuple(R.shape), dtype=torch.float32, device=R.device)
        V[0] = (Rc / col(torch.tensor(np.where(beta > 0, beta, 1.0), device=R.device))).float()
        H = np.zeros((k, m + 1, m))
        cs, sn = np.zeros((k, m)), np.zeros((k, m))
        g = np.zeros((k, m + 1))
        g[:, 0] = beta
        j_used = 0
        for j in range(m):
            apply(V[j], W)
            w = W
            for i in range(j + 1):  # modified Gram-Schmidt, fp64 accumulation of fp32 vectors
                h = (V[i].double() * w).sum(rd)
                w = w - col(h) * V[i].double()
                H[:, i, j] = h.cpu().numpy()
            hn = torch.linalg.norm(w, dim=rd)
            H[:, j + 1, j] = hn.cpu().numpy()
            V[j + 1] = (w / col(torch.where(hn > 0, hn, torch.ones_like(hn)))).float()
            for r in range(k):  # Givens (gmres.cpp:120-150) per right-hand side
                for i in range(j):
                    t = cs[r, i] * H[r, i, j] + sn[r, i] * H[r, i + 1, j]
                    H[r, i + 1, j] = -sn[r, i] * H[r, i, j] + cs[r, i] * H[r, i + 1, j]
                    H[r, i, j] = t
                a, b = H[r, j, j], H[r, j + 1, j]
                den = np.hypot(a, b)
                cs[r, j], sn[r, j] = (1.0, 0.0) if den == 0 else (a / den, b / den)
                H[r, j, j] = cs[r, j] * a + sn[r, j] * b
                H[r, j + 1, j] = 0.0
                g[r, j + 1] = -sn[r, j] * g[r, j]
                g[r, j] = cs[r, j] * g[r, j]
            its += 1
            j_used = j + 1
            if (np.abs(g[:, j + 1]) <= tol * r0).all():
                break
        Y = np.zeros((k, j_used))
        for r in range(k):
            if done[r]:
                continue
            Hr = np.triu(H[r, :j_used, :j_used])
            try:
                Y[r] = np.linalg.solve(Hr, g[r, :j_used])
            except np.linalg.LinAlgError:  # breakdown: least squares on the rotated system
                Y[r] = np.linalg.lstsq(Hr, g[r, :j_used], rcond=None)[0]
        Yt = torch.tensor(Y, device=R.device)
        if rd == 1:
            D += torch.einsum("kj,jkn->kn", Yt, V[:j_used].double())
        else:
            D += torch.einsum("kj,jnk->nk", Yt, V[:j_used].double())
    return D, its


def gmres_mixed(op, B, tol=1e-12, m=40, inner_tol=1e-6, max_outer=30, max_cycles=20, fp32_op=None, fp64_mfma=None,
                native=None):
    """Solve A X = B (rows) to ||B - A X|| / ||B|| <= tol per row.  Returns
    (X, outer iterations, inner iterations, final relative residuals).

    native (default: 16 rows on a handle with the library solve, both MFMA operators):
    the whole solve runs in the library (Aniso.solve16_mixed_dev,
    aniso_solve16_mixed_dev: the same refinement and inner GMRES with the DCGS2
    Arnoldi of the block solve on an fp32 basis, no torch op and no host round trip
    inside a step).  native=False keeps the torch-orchestrated loop below (the
    reference the library's solve is tested against).

    fp32_op (default: when B has 16 rows): the inner solves run on the fp32 MFMA
    operator (Aniso.forward_f32_dev, fp32 caches) in tree order, point-major; the
    outer residuals stay in fp64, so the solution is fp64-accurate.
    fp64_mfma (default: when B has 16 rows): the outer fp64 residuals run on the fp64
    MFMA operator (Aniso.forward16_f64_dev) instead of two 8-row VALU batches."""
    import torch

    if fp32_op is None:
        fp32_op = B.shape[0] == 16
    if fp64_mfma is None:
        fp64_mfma = B.shape[0] == 16 and hasattr(op, "forward16_f64_dev")
    if native is None:
        native = fp32_op and fp64_mfma and hasattr(op, "solve16_mixed_dev") and B.is_cuda
    if native:
        X = torch.zeros_like(B)
        outer, inner, rel = op.solve16_mixed_dev(B.contiguous(), X, m=m, tol=tol, inner_tol=inner_tol,
                                                 max_outer=max_outer, max_cycles=max_cycles)
        return X, outer, inner, rel
    X = torch.zeros_like(B)
    W = torch.empty_like(B)
    bn = torch.linalg.norm(B, dim=1)
    inner = 0
    if fp32_op:
        perm = torch.tensor(op.tree_perm(), device=B.device, dtype=torch.int64)
        X32 = torch.empty((B.shape[1], 16), dtype=torch.float32, device=B.device)
        W32 = torch.empty_like(X32)

        def apply32(Xin, Wout):
            X32.copy_(Xin)
            op.forward_f32_dev(X32, W32)
            Wout.copy_(W32)

    if fp64_mfma:
        perm64 = torch.tensor(op.tree_perm(), device=B.device, dtype=torch.int64)
    for outer in range(max_outer + 1):
        if fp64_mfma:
            forward16(op, X, W, perm64)
        else:
            forward_block(op, X, W)
        R = B - W
        rel = (torch.linalg.norm(R, dim=1) / bn).cpu().numpy()
        if (rel <= tol).all() or outer == max_outer:
            return X, outer, inner, rel
        if fp32_op:
            D, its = _inner_gmres(apply32, R[:, perm].t().contiguous(), m, inner_tol, max_cycles, rd=0)
            X[:, perm] += D.t()
        else:
            D, its = _inner_gmres(lambda a, b: forward_block(op, a.double(), b), R, m, inner_tol, max_cycles)
            X += D
        inner += its
    return X, max_outer, inner, rel


def gmres_dist(apply, b, restart=400, tol=1e-11, maxit=400, x0=None, allreduce=None, hist=None, kry=None):
    """Restarted GMRES with MATLAB's semantics (aniso.m:159-173: gmres(A, rhs, restart,
    tol, maxit); the Arnoldi/Givens structure of gmres.cpp:53-169) on vectors that may
    be row slices of a sharded problem.

    apply(x, y): y = A x on this rank's slice (the caller's operator does its own
    exchanges: the sharded block matvec's halo all-to-all and root all-gather).
    allreduce(t): sums a small float64 tensor over the ranks in place (None: one rank).
    Orthogonalisation is classical Gram-Schmidt with one reorthogonalisation (CGS2):
    each Arnoldi step reduces its inner products in TWO all-reduces -- [V^T w] and
    [V^T w', w'.w'] -- instead of the j + 1 dependent reductions of modified
    Gram-Schmidt (gmres.cpp:116-120), which would put j latency-bound collectives
    on every step.  Converged when ||b - A x|| / ||b|| <= tol (the estimate inside a
    cycle, confirmed by the explicit residual at its end).

    Returns (x, total steps (negative if not converged), final relative residual).
    hist (a list) receives the estimate after every step.

    kry (an aniso_amd.Aniso handle, CUDA vectors): the Arnoldi process runs on the
    library's DCGS2 primitives (aniso_arnoldi_*: two sweeps over the basis per step,
    Hessenberg matrix, rotations and residual estimate on the device; with allreduce,
    the step's two sets of inner products are summed over the ranks between its
    parts), and the next step's matvec is enqueued before the host reads the step's
    residual estimate (except where it is predicted to reach tol)."""
    import torch

    red = allreduce or (lambda t: t)
    x = torch.zeros_like(b) if x0 is None else x0.clone()
    w = torch.empty_like(b)
    n = b.numel()

    def nrm(v):
        t = (v.reshape(-1) @ v.reshape(-1)).reshape(1)
        red(t)
        return float(t.sqrt())

    def residual():
        apply(x, w)
        return b - w

    normb = nrm(b)
    if normb == 0.0:
        return torch.zeros_like(b), 0, 0.0
    m = restart
    V = torch.empty((m + 1, n), dtype=b.dtype, device=b.device)
    if kry is not None:
        return _gmres_dist_dev(apply, b, x, w, V, m, tol, maxit, allreduce, normb, x0 is None, hist, kry)
    r = residual()
    beta = nrm(r)
    relres = beta / normb
    total = 0
    for _ in range(maxit):
        if relres <= tol or beta == 0.0:
            break
        V[0] = r.reshape(-1) / beta
        H = np.zeros((m + 1, m))
        cs, sn, g = np.zeros(m), np.zeros(m), np.zeros(m + 1)
        g[0] = beta
        used = 0
        for i in range(m):
            apply(V[i].view_as(b), w)
            wv = w.reshape(-1).clone()
            Vi = V[: i + 1]
            h = Vi @ wv
            red(h)
            wv -= Vi.t() @ h
            h2 = torch.cat([Vi @ wv, (wv @ wv).reshape(1)])
            red(h2)
            wv -= Vi.t() @ h2[: i + 1]
            h = (h + h2[: i + 1]).cpu().numpy()
            hn = float(max(h2[i + 1] - h2[: i + 1] @ h2[: i + 1], 0.0)) ** 0.5
            H[: i + 1, i] = h
            H[i + 1, i] = hn
            V[i + 1] = wv / hn if hn > 0 else 0.0
            for k in range(i):  # the previous rotations (gmres.cpp:136-139)
                t = cs[k] * H[k, i] + sn[k] * H[k + 1, i]
                H[k + 1, i] = -sn[k] * H[k, i] + cs[k] * H[k + 1, i]
                H[k, i] = t
            den = np.hypot(H[i, i], H[i + 1, i])
            cs[i], sn[i] = (1.0, 0.0) if den == 0 else (H[i, i] / den, H[i + 1, i] / den)
            H[i, i], H[i + 1, i] = den, 0.0
            g[i + 1] = -sn[i] * g[i]
            g[i] = cs[i] * g[i]
            total += 1
            used = i + 1
            relres = abs(g[i + 1]) / normb
            if hist is not None:
                hist.append(relres)
            if relres <= tol or hn == 0.0:
                break
        y = np.zeros(used)
        for k in range(used - 1, -1, -1):
            y[k] = (g[k] - H[k, k + 1:used] @ y[k + 1:]) / H[k, k] if H[k, k] != 0 else 0.0
        x += (V[:used].t() @ torch.tensor(y, dtype=b.dtype, device=b.device)).view_as(b)
        r = residual()
        beta = nrm(r)
        relres = beta / normb
    return x, (total if relres <= tol else -max(total, 1)), relres


def _gmres_dist_dev(apply, b, x, w, V, m, tol, maxit, allreduce, normb, x_zero, hist, kry):
    """gmres_dist's loop on the library's DCGS2 primitives (see gmres_dist: kry).  V[0]
    holds each cycle's residual; the stored vectors are never rewritten (arnoldi.hpp)."""
    import torch

    from . import MappedStatus

    n = b.numel()
    st = kry.arnoldi_state(m)
    # the status word: one pinned mapped allocation per handle, reused by its solves
    stat = getattr(kry, "_gmres_status", None)
    if stat is None:
        stat = kry._gmres_status = MappedStatus(4)
    out = torch.zeros(m + 2, dtype=torch.float64, device=b.device)
    ev = torch.cuda.Event()
    bv, wv, xv = b.reshape(-1), w.reshape(-1), x.reshape(-1)
    total, relres = 0, 1.0

    def begin():  # r = b - A x into V[0], the cycle's start; (|r| / |b|, |r|)
        if x_zero:
            V[0].copy_(bv)
        else:
            apply(x, w)
            torch.sub(bv, wv, out=V[0])
        if allreduce is None:
            kry.arnoldi_begin(V, m, st, normb, status=stat)
        else:  # this rank's |r|^2 in the one-rank path's summation order, then summed over the ranks
            kry.arnoldi_project(V, 0, V[0], out)
            allreduce(out[:1])
            kry.arnoldi_begin(V, m, st, normb, rr=out, status=stat)
        ev.record()
        ev.synchronize()
        return float(stat.host[0]), float(stat.host[1])

    try:
        for _ in range(maxit):
            relres, rnorm = begin()
            if relres <= tol or rnorm == 0.0:
                break
            used, ahead, hrel = 0, False, []
            for j in range(m):
                if not ahead:
                    apply(V[j].view_as(b), w)
                if allreduce is None:
                    kry.arnoldi_step(V, m, j, wv, st, status=stat)
                else:
                    kry.arnoldi_project(V, j, wv, out)
                    allreduce(out[: j + 1])
                    kry.arnoldi_coef(m, j, st, out)
                    kry.arnoldi_update(V, m, j, wv, st, out)
                    allreduce(out[: j + 2])
                    kry.arnoldi_column(m, j, st, out, status=stat)
                ev.record()
                # the next matvec runs while the host reads this step's estimate, unless
                # that estimate is predicted to reach tol (the last two estimates' ratio,
                # 10x margin)
                near = False
                if len(hrel) >= 2:
                    near = hrel[-1] * min(1.0, hrel[-1] / hrel[-2]) <= 10.0 * tol
                elif hrel:
                    near = hrel[-1] <= 10.0 * tol
                ahead = j + 1 < m and not near
                if ahead:
                    apply(V[j + 1].view_as(b), w)
                ev.synchronize()
                rel, rn = float(stat.host[0]), float(stat.host[1])
                total += 1
                used = j + 1
                relres = rel
                hrel.append(rel)
                if hist is not None:
                    hist.append(rel)
                if rel <= tol or rn == 0.0:
                    break
            kry.arnoldi_solution(V, m, used, st, xv)
            x_zero = x_zero and used == 0
        else:
            relres, _ = begin()
    finally:
        torch.cuda.synchronize()  # no kernel may still write the reused status word
    return x, (total if relres <= tol else -max(total, 1)), relres
