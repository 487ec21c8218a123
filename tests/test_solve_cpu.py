"""CPU checks of the multi-RHS mixed-precision GMRES driver (aniso_amd/solve.py) on a
dense stand-in operator with the same call shape as Aniso.apply_block_dev, and of the
config-5 centre generator (std::mt19937_64)."""
import numpy as np
import torch

from aniso_amd.solve import MT19937_64, config5_charges, gmres_mixed


class DenseOp:
    """K x with sigma: apply_block_dev(x, ids, mixes, out, use_sigma) -> out = mix (K (sig x))."""

    def __init__(self, n, seed):
        rng = np.random.default_rng(seed)
        self.K = torch.tensor(rng.uniform(-1, 1, (n, n)) / (2.5 * np.sqrt(n)))
        self.sig = torch.tensor(rng.uniform(0.5, 1.0, n))
        self.perm = rng.permutation(n).astype(np.int32)

    def apply_block_dev(self, x, ids, mixes, out, use_sigma=False):
        y = (x * self.sig if use_sigma else x) @ self.K.T
        out.copy_(torch.tensor(mixes[0]) @ y)

    def tree_perm(self):
        return self.perm

    def forward16_f64_dev(self, X, Y):
        """The fp64 MFMA operator's call shape: (n, 16) float64, tree order, point-major."""
        K = self.K[self.perm][:, self.perm]
        s = self.sig[self.perm]
        Y.copy_(X - K @ (s[:, None] * X))

    def forward_f32_dev(self, X, Y):
        """The fp32 operator's call shape: (n, 16) float32, tree order, point-major."""
        K = self.K[self.perm][:, self.perm].float()
        s = self.sig[self.perm].float()
        Y.copy_(X - K @ (s[:, None] * X))


def test_mt19937_64_reference_value():
    g = MT19937_64(5489)
    for _ in range(9999):
        g()
    assert g() == 9981545732273789042  # the C++ standard's check value


def test_config5_charges_are_gaussian_bumps_in_the_box():
    xy = np.random.default_rng(0).uniform(0, 1, (500, 2))
    for k in range(16):
        q = config5_charges(xy, k)
        c = xy[np.argmax(q)]
        assert q.max() <= 1.0 and q.min() > 0.0
        assert 0.1 <= c[0] <= 0.9 and 0.1 <= c[1] <= 0.9


import pytest  # noqa: E402


@pytest.mark.parametrize("fp32_op,fp64_mfma", [(True, True), (False, False), (True, False)])
def test_mixed_gmres_matches_dense_solve_for_16_rhs(fp32_op, fp64_mfma):
    """Both inner operators: the fp32 one (tree order, point-major, as
    Aniso.forward_f32_dev) and the fp64 row-layout one; the outer fp64 residual
    through the 16-RHS operator's layout (Aniso.forward16_f64_dev) or the rows."""
    n, k = 300, 16
    op = DenseOp(n, 1)
    A = np.eye(n) - op.K.numpy() * op.sig.numpy()[None, :]
    B = torch.tensor(np.random.default_rng(2).uniform(-1, 1, (k, n)))
    X, outer, inner, rel = gmres_mixed(op, B, tol=1e-12, m=30, inner_tol=1e-6, fp32_op=fp32_op, fp64_mfma=fp64_mfma)
    ref = np.linalg.solve(A, B.numpy().T).T
    assert (rel <= 1e-12).all() and outer >= 2  # fp32 inner solves need refinement
    assert np.linalg.norm(X.numpy() - ref) / np.linalg.norm(ref) <= 1e-10
