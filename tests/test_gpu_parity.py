"""Parity of the HIP path (through the C ABI) against the CPU oracle, the
reference's recorded known answers, and size-independent properties.

Tolerance (BASELINE.json north_star: "<= 1e-10 relative error"): relative L2 error
<= 1e-10 of every full apply; per-stage errors are measured against the norm of
the full output (a stage can be ~0, e.g. odd modes' singular term at d=1).
"""
import json
import os

import numpy as np
import pytest

from conftest import gaussian_charge, main_coeffs, rough_coeffs

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KA = json.load(open(os.path.join(ROOT, "tests", "golden", "survey_known_answers.json")))
TOL = 1e-10


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _pair(sz, d, ks, ns, ml=20, coeffs="main", seed=0):
    import aniso_amd
    from oracle.oracle_py import Oracle

    a = aniso_amd.Aniso(sz, d, ks, 0.8, ns, 4, ml)
    o = Oracle(sz, d, ks, 0.8, ns, 4, ml)
    xy = a.getNodes()
    ss, st = main_coeffs(xy) if coeffs == "main" else rough_coeffs(xy, seed)
    a.setCoeff(ss, st)
    o.setCoeff(ss, st)
    return a, o, xy


CASES = [
    # sz, d, ks, ns, maxLevel, coeffs, modes
    (16, 3, 1, 8, 20, "main", [0]),          # config 1 geometry (data.cfg parameters)
    (8, 1, 5, 10, 20, "main", range(9)),     # aniso.m parameters, all 9 Fourier modes
    (12, 2, 2, 8, 20, "rough", [0, 1, 2]),
    (20, 3, 2, 8, 20, "rough", [0, 2]),
    (11, 3, 1, 6, 20, "rough", [0]),         # odd sz: non-power-of-two tree with W/X lists
    (24, 1, 3, 10, 2, "rough", [0, 3]),      # maxLevel-limited: 64-point leaves
    (8, 2, 1, 8, 0, "main", [0]),            # maxLevel 0: one 256-point leaf, near field only
    (1, 3, 1, 8, 20, "main", [0]),           # single square: the root is the only leaf
    (15, 3, 2, 8, 2, "rough", [0, 1]),       # ~127-point leaves: symmetric and directed U pairs mixed
    (12, 2, 2, 8, 0, "main", [0, 1]),        # one 576-point leaf, directed near: > 64 row quads per wave
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"sz{c[0]}d{c[1]}ks{c[2]}ml{c[4]}{c[5]}")
def test_mapping_matches_oracle(case):
    sz, d, ks, ns, ml, coeffs, modes = case
    a, o, xy = _pair(sz, d, ks, ns, ml, coeffs, seed=sz)
    rng = np.random.default_rng(sz * 31 + d)
    for q in (rng.uniform(-1, 1, a.N), gaussian_charge(xy)):
        for m in modes:
            a.cache(m)
            o.cache(m)
            out = a.mapping(q, m)
            ref = o.mapping(q, m)
            assert _rel(out, ref) <= TOL, (case, m, _rel(out, ref))


@pytest.mark.parametrize("case", CASES[:4], ids=lambda c: f"sz{c[0]}d{c[1]}ks{c[2]}")
def test_stages_match_oracle(case):
    import aniso_amd

    torch = _torch()
    sz, d, ks, ns, ml, coeffs, modes = case
    a, o, xy = _pair(sz, d, ks, ns, ml, coeffs, seed=1)
    q = np.random.default_rng(5).uniform(-1, 1, a.N)
    qd = torch.tensor(q, device="cuda")
    s = 1.0 / (2 * np.pi)
    for m in modes:
        a.cache(m)
        o.cache(m)
        st = o.mapping_stages(q, m)
        ref_total = st[5]
        for mask, ref in ((aniso_amd.STAGE_FAR | aniso_amd.STAGE_NEAR, (st[0] + st[1]) * s),
                          (aniso_amd.STAGE_STENCIL, (st[2] + st[3]) * s),
                          (aniso_amd.STAGE_SING, st[4] * s)):
            od = torch.zeros(a.N, dtype=torch.float64, device="cuda")
            a.mapping_dev(qd, m, od, mask=mask)
            torch.cuda.synchronize()
            err = np.linalg.norm(od.cpu().numpy() - ref) / np.linalg.norm(ref_total)
            assert err <= TOL, (case, m, mask, err)


@pytest.mark.parametrize("name", ["probe256_d1", "probe1M_d3"])
def test_reference_known_answers(name):
    """Full-size pins: outputs the survey recorded from the reference itself."""
    import aniso_amd

    c = [x for x in KA["applies"] if x["name"] == name][0]
    a = aniso_amd.Aniso(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    a.cache(c["mode"])
    out = a.mapping(gaussian_charge(xy), c["mode"])
    assert abs(np.linalg.norm(out) - c["out_norm2"]) <= TOL * c["out_norm2"]
    assert abs(out[0] - c["out0"]) <= TOL * abs(c["out0"])
    assert abs(out[len(out) // 2] - c["outHalf"]) <= 1e-9 * abs(c["outHalf"])


def test_tree_counts_match_reference_at_full_size():
    import aniso_amd

    for c in KA["trees"]:
        a = aniso_amd.Aniso(c["sz"], c["d"], 1, 0.5, 8, c["np"], c["maxLevel"])
        s = a.stats()
        assert s["tree_nodes"] == c["nodes"] and s["near_entries"] == c["nearPairs"]
        assert s["m2l_entries"] == c["M2Lpairs"], c["name"]


def test_line_integrals_match_oracle():
    a, o, xy = _pair(17, 3, 1, 8, 20, "rough", seed=9)
    rng = np.random.default_rng(11)
    seg = rng.uniform(0.001, 0.999, (4000, 4))
    seg[:500, 2] = seg[:500, 0]          # vertical segments
    seg[500:1000, 3] = seg[500:1000, 1]  # horizontal segments
    seg[1000:1100, 2:] = seg[1000:1100, :2] + 1e-3 * rng.uniform(-1, 1, (100, 2))  # short
    k = np.arange(1, 16) / 17.0          # through grid corners
    seg[1100:1115] = np.stack([k * 0 + 0.01, k * 0 + 0.01, k, k], 1)
    got = a.line_integrals(seg)
    ref = np.array([o.line_integral(*s) for s in seg])
    assert np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))) <= 1e-12


def test_linearity_and_determinism_at_config3_size():
    """Size-independent properties at BASELINE's 1M-point geometry (config 3)."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(1024, 1, 1, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    a.cache(0)
    rng = np.random.default_rng(1)
    q1 = torch.tensor(rng.uniform(-1, 1, a.N), device="cuda")
    q2 = torch.tensor(gaussian_charge(xy), device="cuda")
    o1, o2, o3, o4 = (torch.zeros_like(q1) for _ in range(4))
    a.mapping_dev(q1, 0, o1)
    a.mapping_dev(q2, 0, o2)
    a.mapping_dev(2.5 * q1 - 0.75 * q2, 0, o3)
    a.mapping_dev(q1, 0, o4)
    torch.cuda.synchronize()
    lin = 2.5 * o1 - 0.75 * o2
    assert float(torch.linalg.norm(o3 - lin) / torch.linalg.norm(lin)) <= 1e-13
    assert torch.equal(o1, o4)  # bitwise deterministic
    # positive kernel: a positive charge gives a positive potential
    assert float(o2.min()) > 0


@pytest.mark.parametrize("nranks", [2, 3])
def test_sharded_apply_composes_to_full(nranks):
    torch = _torch()
    import aniso_amd
    from aniso_amd import dist as adist

    sz, d, ks = 40, 2, 2
    full = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 4)
    full.setCoeff(*coef)
    full.cache(1)
    q = torch.tensor(np.random.default_rng(2).uniform(-1, 1, full.N), device="cuda")
    ref = torch.zeros_like(q)
    full.mapping_dev(q, 1, ref)
    ranges = adist.shard_ranges(full, nranks)
    perm = torch.tensor(full.tree_perm(), device="cuda", dtype=torch.int64)
    got = torch.zeros_like(q)
    for r in range(nranks):
        sh = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
        sh.set_shard(r, nranks)
        sh.setCoeff(*coef)
        sh.cache(1)
        out = torch.full_like(q, float("nan"))
        sh.mapping_dev(q, 1, out)  # writes only the shard's own targets (original order)
        own = perm[ranges[r][0]:ranges[r][1]]
        got[own] = out[own]
    torch.cuda.synchronize()
    assert float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref)) <= 1e-14


def test_batched_and_device_variants_agree():
    torch = _torch()
    a, o, xy = _pair(10, 2, 1, 8, 20, "rough", seed=3)
    a.cache(0)
    Q = np.random.default_rng(4).uniform(-1, 1, (a.N, 3))
    B = a.mapping_batched(Q, 0)
    for j in range(3):
        assert np.array_equal(B[:, j], a.mapping(Q[:, j], 0))
    qd = torch.tensor(Q[:, 0], device="cuda")
    od = torch.zeros_like(qd)
    a.mapping_dev(qd, 0, od)
    torch.cuda.synchronize()
    assert np.array_equal(od.cpu().numpy(), B[:, 0])


def test_forward_operator_and_gmres_match_reference():
    """main.cpp's GMRES on the device: same iteration count as the reference
    (29 for the literal data.cfg) and the same solution as the oracle's GMRES."""
    torch = _torch()
    import aniso_amd
    from oracle.oracle_py import Oracle

    c = KA["gmres"][0]
    a = aniso_amd.Aniso(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    xy = a.getNodes()
    ss, st = main_coeffs(xy)
    a.setCoeff(ss, st)
    a.cache(0)
    q = gaussian_charge(xy)
    # forward operator u - K0(sigma_s u)
    u = torch.tensor(np.random.default_rng(0).uniform(-1, 1, a.N), device="cuda")
    f = torch.zeros_like(u)
    a.forward_dev(u, f)
    k = a.mapping(u.cpu().numpy() * ss, 0)
    torch.cuda.synchronize()
    assert np.allclose(f.cpu().numpy(), u.cpu().numpy() - k, rtol=0, atol=1e-13 * np.abs(k).max())
    j, x, hist, fr = a.gmres(q, c["m"], c["maxit"], c["tol"])
    assert j == c["iterations"], (j, hist)
    assert fr < c["tol"]
    o = Oracle(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    o.setCoeff(ss, st)
    o.cache(0)
    jo, xo, ho, fro = o.gmres_main(q, c["m"], c["maxit"], c["tol"])
    assert jo == j
    assert _rel(x, xo) <= 1e-10
    # residual histories agree until rounding noise (~1e-16 |b|) dominates the residual
    assert np.allclose(hist, ho[: len(hist)], rtol=1e-4, atol=1e-15)


def test_uncached_mode_fails_loudly():
    import aniso_amd

    a = aniso_amd.Aniso(6, 1, 2, 0.8, 8, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    a.cache(0)
    with pytest.raises(aniso_amd.AnisoError) as e:
        a.mapping(np.ones(a.N), 2)
    assert e.value.code == 3


@pytest.mark.parametrize("comm,port", [("native", 29533), ("python", 29534), ("native", None)])
def test_bench_sharded_path_rehearsal_two_ranks(comm, port):
    """bench.py's N>1 matvec (subtree shards, halo all-to-all, root all-gather) with
    two ranks sharing the one GPU of the box over gloo: through the library's own
    exchange (one C call per matvec, aniso_comm_init_callbacks) and through
    aniso_amd.dist.ShardExchange; each rank's input holds only its own range (native)
    or own range + halo (python), NaN elsewhere; checked against the unsharded op,
    with the GMRES leg over the shards.  port None: `bench.py --gpus 2` run bare, the
    way the driver may call it -- bench.py starts its two ranks itself."""
    import subprocess
    import sys

    launcher = [] if port is None else [
        "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
        f"--master-port={port}"]
    cmd = [sys.executable] + launcher + [
        os.path.join(ROOT, "bench.py"),
        "--gpus", "2", "--steps", "2", "--warmup", "1", "--sz", "128", "--backend", "gloo",
        "--same-device", "--verify", "--no-cpu", "--comm", comm, "--gmres", "6", "--config4-sz", "256"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2
    assert res["verify_rel_err_vs_unsharded"] <= 1e-13
    assert res["verify_halo_rel_err"] <= 1e-15
    assert res["gmres"]["steps"] == 6 and res["gmres"]["relres_after"] < 1.0
    assert res["config4"]["N"] == 256 * 256 and res["config4"]["matvec_per_s"] > 0


def test_rccl_shard_exchange_collectives_one_rank():
    """ShardExchange's all-gather and halo all-to-all through RCCL (backend "nccl"),
    one rank on the box's GPU (tools/rccl_check.py): the calls bench.py makes at N > 1."""
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=29537", os.path.join(ROOT, "tools", "rccl_check.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert res["allgather_equal"] and res["halo_equal"] and res["empty_halo_untouched"]


@pytest.mark.parametrize("sz,d,ks,ml", [(32, 1, 2, 20), (11, 3, 2, 20), (15, 3, 2, 2)])
def test_symmetric_storage_matches_directed(sz, d, ks, ml, monkeypatch):
    """Symmetric M2L / U-pair storage against the fully directed
    plan (ANISO_SYMMETRIC=0) and the oracle, for even and odd modes."""
    import aniso_amd

    _torch()
    monkeypatch.setenv("ANISO_NEAR_SYMMETRIC", "1")
    a, o, xy = _pair(sz, d, ks, 8, ml, "rough", seed=3)
    monkeypatch.delenv("ANISO_NEAR_SYMMETRIC")
    monkeypatch.setenv("ANISO_SYMMETRIC", "0")
    b = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, ml)
    monkeypatch.delenv("ANISO_SYMMETRIC")
    b.setCoeff(*rough_coeffs(xy, 3))
    sa, sb = a.stats(), b.stats()
    assert sa["m2l_canon"] > 0 and sb["m2l_canon"] == 0 and sb["near_partial"] == 0
    assert sa["stored_m2l"] < sb["stored_m2l"] and sa["stored_near"] < sb["stored_near"]
    assert sa["m2l_pairs"] == sb["m2l_pairs"] and sa["near_entries"] == sb["near_entries"]
    q = np.random.default_rng(5).uniform(-1, 1, a.N)
    for m in range(2 * ks - 1):
        for x in (a, b, o):
            x.cache(m)
        ya, yb, yo = a.mapping(q, m), b.mapping(q, m), o.mapping(q, m)
        assert _rel(ya, yb) <= 1e-12, (m, _rel(ya, yb))
        assert _rel(ya, yo) <= TOL and _rel(yb, yo) <= TOL


@pytest.mark.parametrize("nranks", [1, 3])
def test_tree_order_paths_match_original_order(nranks):
    """aniso_mapping_tree_dev / aniso_forward_tree_dev (tree-order vectors, owned
    slices) against the original-order apply and forward operator, unsharded and
    composed over shards by concatenating their owned tree-order slices."""
    torch = _torch()
    import aniso_amd
    from aniso_amd import dist as adist

    sz, d, ks = 24, 3, 2
    full = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 9)
    full.setCoeff(*coef)
    full.cache(0)
    full.cache(1)
    perm = torch.tensor(full.tree_perm(), device="cuda", dtype=torch.int64)
    q = torch.tensor(np.random.default_rng(3).uniform(-1, 1, full.N), device="cuda")
    ref1 = torch.zeros_like(q)
    full.mapping_dev(q, 1, ref1)
    reff = torch.zeros_like(q)
    full.forward_dev(q, reff)
    ranges = adist.shard_ranges(full, nranks)
    qt = q[perm].contiguous()
    s1, sf = [], []
    for r in range(nranks):
        sh = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
        sh.set_shard(r, nranks)
        sh.setCoeff(*coef)
        sh.cache(0)
        sh.cache(1)
        n = ranges[r][1] - ranges[r][0]
        s1.append(torch.zeros(n, dtype=torch.float64, device="cuda"))
        sf.append(torch.zeros(n, dtype=torch.float64, device="cuda"))
        sh.mapping_tree_dev(qt, 1, s1[-1])
        sh.forward_tree_dev(qt, sf[-1])
        torch.cuda.synchronize()
    got1 = torch.cat(s1)
    gotf = torch.cat(sf)
    assert float(torch.linalg.norm(got1 - ref1[perm]) / torch.linalg.norm(ref1)) <= 1e-14
    assert float(torch.linalg.norm(gotf - reff[perm]) / torch.linalg.norm(reff)) <= 1e-14


def _block_ref(o, U, g, ss, which):
    """aniso.m forward / mforward / x - mforward(x) composed from oracle mode applies."""
    nb = U.shape[0]
    out = np.zeros_like(U)
    memo = {}
    for i in range(-(nb - 1), 1):
        iid = abs(i)
        for j in range(-(nb - 1), nb):
            b, m = abs(j), abs(i - j)
            if (b, m) not in memo:
                memo[(b, m)] = o.mapping(U[b] * ss if which else U[b], m)
            w = (g ** b - g ** nb) / (1 - g ** nb) if which else 1.0
            out[iid] += w * memo[(b, m)]
    return U - out if which == 2 else out


@pytest.mark.parametrize("sz,d,ks,coeffs", [(12, 1, 5, "main"), (10, 2, 3, "rough"), (9, 3, 2, "rough")])
def test_block_operator_matches_oracle(sz, d, ks, coeffs):
    """aniso.m's forward, mforward and GMRES matvec x - mforward(x) (one batched
    apply over all 2ks-1 modes) against the oracle's per-mode applies."""
    torch = _torch()
    a, o, xy = _pair(sz, d, ks, 8, 20, coeffs, seed=7)
    ss = main_coeffs(xy)[0] if coeffs == "main" else rough_coeffs(xy, 7)[0]
    for m in range(2 * ks - 1):
        a.cache(m)
        o.cache(m)
    U = np.random.default_rng(sz).uniform(-1, 1, (ks, a.N))
    U[0] += gaussian_charge(xy)
    Ud = torch.tensor(U, device="cuda")
    for which in (0, 1, 2):
        out = torch.zeros_like(Ud)
        a.block_op_dev(which, Ud, out)
        torch.cuda.synchronize()
        ref = _block_ref(o, U, a.g, ss, which)
        assert _rel(out.cpu().numpy(), ref) <= TOL, (which, _rel(out.cpu().numpy(), ref))
        # the host-pointer boundary (aniso_block_op; the MEX shim's forward /
        # mforward / blockMatvec ops): stacked aniso.m column in, same result
        host = a.block_op(which, U.reshape(-1))
        assert _rel(host, ref) <= TOL, (which, _rel(host, ref))
    # SURVEY.md §8b aniso_apply_block(h, u, sigma_s, g, out): explicit sigma_s and g,
    # both different from the handle's (the caches depend on sigma_t only)
    ss2 = ss * 0.5 + 0.25
    ref = _block_ref(o, U, 0.6, ss2, 2)
    host = a.apply_block(U, ss2, 0.6)
    assert _rel(host, ref) <= TOL, _rel(host, ref)
    # ... and the handle's own sigma_s / g again afterwards (no state leaks)
    assert _rel(a.block_op(2, U), _block_ref(o, U, a.g, ss, 2)) <= TOL


@pytest.mark.parametrize("nrhs,near_sym", [(1, 0), (2, 0), (3, 0), (4, 0), (5, 0), (6, 0), (8, 0), (2, 1), (5, 1)])
def test_apply_block_generic_mixes(nrhs, near_sym, monkeypatch):
    """Arbitrary mixes and mode terms, every right-hand-side count (3, 6 pad to 4, 8),
    strided input/output rows, with and without sigma_s; directed and symmetric
    near-field storage."""
    torch = _torch()
    monkeypatch.setenv("ANISO_NEAR_SYMMETRIC", str(near_sym))
    a, o, xy = _pair(11, 2, 3, 8, 20, "rough", seed=2)
    assert (a.stats()["near_partial"] > 0) == bool(near_sym)
    ss = rough_coeffs(xy, 2)[0]
    ids = [0, 3, 1]
    for m in ids:
        a.cache(m)
        o.cache(m)
    rng = np.random.default_rng(nrhs)
    X = rng.uniform(-1, 1, (nrhs, a.N))
    mixes = rng.uniform(-1, 1, (len(ids), nrhs, nrhs))
    xbuf = torch.zeros(nrhs, a.N + 13, dtype=torch.float64, device="cuda")
    xbuf[:, :a.N] = torch.tensor(X, device="cuda")
    for use_sigma in (False, True):
        obuf = torch.full((nrhs, a.N + 5), 7.0, dtype=torch.float64, device="cuda")
        a.apply_block_dev(xbuf[:, :a.N], ids, mixes, obuf[:, :a.N], use_sigma=use_sigma)
        torch.cuda.synchronize()
        base = [[o.mapping(X[b] * ss if use_sigma else X[b], m) for b in range(nrhs)] for m in ids]
        ref = np.zeros((nrhs, a.N))
        for t in range(len(ids)):
            for i in range(nrhs):
                for b in range(nrhs):
                    ref[i] += mixes[t, i, b] * base[t][b]
        got = obuf.cpu().numpy()
        assert _rel(got[:, :a.N], ref) <= TOL, (nrhs, use_sigma, _rel(got[:, :a.N], ref))
        assert np.all(got[:, a.N:] == 7.0)  # padding columns untouched


def test_block_matvec_tree_order_and_shards_compose():
    """The multi-GPU form of the block matvec: tree-order input, owned slices out,
    per-shard handles whose slices concatenate to the unsharded result."""
    torch = _torch()
    import aniso_amd

    sz, d, ks = 24, 2, 3
    full = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 5)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    perm = torch.tensor(full.tree_perm(), device="cuda", dtype=torch.int64)
    U = torch.tensor(np.random.default_rng(3).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(U)
    full.block_op_dev(2, U, ref)
    Ut = U[:, perm].contiguous()
    tree_out = torch.zeros_like(U)
    full.block_op_dev(2, Ut, tree_out, tree=True)
    torch.cuda.synchronize()
    assert float(torch.linalg.norm(tree_out - ref[:, perm]) / torch.linalg.norm(ref)) <= 1e-14
    parts = []
    for r in range(3):
        sh = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
        sh.set_shard(r, 3)
        sh.setCoeff(*coef)
        for m in range(2 * ks - 1):
            sh.cache(m)
        b, e = sh.shard()
        part = torch.zeros(ks, e - b, dtype=torch.float64, device="cuda")
        sh.block_op_dev(2, Ut, part, tree=True)
        parts.append(part)
    torch.cuda.synchronize()
    got = torch.cat(parts, 1)
    assert float(torch.linalg.norm(got - ref[:, perm]) / torch.linalg.norm(ref)) <= 1e-14


def test_block_matvec_at_config3_size_matches_mode_applies():
    """At BASELINE's 1M-point geometry (config 3: g = 0.8, 9 modes x 5 blocks): the
    batched block matvec equals its composition from 45 single-mode device applies,
    and repeats to rounding."""
    torch = _torch()
    import aniso_amd

    ks, g = 5, 0.8
    a = aniso_amd.Aniso(1024, 1, ks, g, 10, 4, 20)
    xy = a.getNodes()
    ss, st = main_coeffs(xy)
    a.setCoeff(ss, st)
    for m in range(2 * ks - 1):
        a.cache(m)
    U = torch.tensor(np.random.default_rng(9).uniform(-1, 1, (ks, a.N)), device="cuda")
    y1, y2 = torch.zeros_like(U), torch.zeros_like(U)
    a.block_op_dev(2, U, y1)
    a.block_op_dev(2, U, y2)
    sd = torch.tensor(ss, device="cuda")
    mix = aniso_amd.block_mixes(ks, g, True)
    ref = U.clone()
    tmp = torch.zeros(a.N, dtype=torch.float64, device="cuda")
    for m in range(2 * ks - 1):
        for b in range(ks):
            if not np.any(mix[m, :, b]):
                continue
            a.mapping_dev((U[b] * sd).contiguous(), m, tmp)
            for i in range(ks):
                if mix[m, i, b]:
                    ref[i] -= float(mix[m, i, b]) * tmp
    torch.cuda.synchronize()
    # the clustered harmonic M2L adds in-cluster products in LDS in arrival order
    # (DESIGN.md §3.10): repeat runs agree to rounding, not bitwise
    assert float(torch.linalg.norm(y1 - y2) / torch.linalg.norm(y1)) <= 1e-15
    assert float(torch.linalg.norm(y1 - ref) / torch.linalg.norm(ref)) <= 1e-13


@pytest.mark.parametrize("sz,d,ks,ml,coeffs", [(16, 1, 5, 20, "main"), (13, 2, 3, 20, "rough"), (20, 1, 2, 20, "rough"),
                                                (11, 3, 4, 20, "rough"), (24, 1, 5, 2, "rough"), (12, 2, 2, 0, "main")])
def test_harmonic_block_apply_matches_per_mode_stream(sz, d, ks, ml, coeffs, monkeypatch):
    """The mode-shared (harmonic) block apply (one read of the
    e^-tau caches for all 2ks-1 modes) against the per-mode operator stream and the
    oracle, for aniso.m's forward / mforward / GMRES matvec; odd sz (X/W lists),
    maxLevel-limited 64-point leaves, a single 576-point leaf (G = 64 lanes per leaf),
    padded block counts (3 -> 4)."""
    torch = _torch()
    import aniso_amd
    from oracle.oracle_py import Oracle

    def make(harmonic):
        monkeypatch.setenv("ANISO_HARMONIC", "1" if harmonic else "0")
        a = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, ml)
        xy = a.getNodes()
        a.setCoeff(*(main_coeffs(xy) if coeffs == "main" else rough_coeffs(xy, 4)))
        for m in range(2 * ks - 1):
            a.cache(m)
        return a, xy

    h, xy = make(True)
    p, _ = make(False)
    assert h.stats()["harmonic"] == 1 and p.stats()["harmonic"] == 0
    o = Oracle(sz, d, ks, 0.8, 8, 4, ml)
    ss, st = main_coeffs(xy) if coeffs == "main" else rough_coeffs(xy, 4)
    o.setCoeff(ss, st)
    for m in range(2 * ks - 1):
        o.cache(m)
    U = np.random.default_rng(ks + sz).uniform(-1, 1, (ks, h.N))
    U[0] += gaussian_charge(xy)
    Ud = torch.tensor(U, device="cuda")
    for which in (0, 1, 2):
        oh, op_ = torch.zeros_like(Ud), torch.zeros_like(Ud)
        h.block_op_dev(which, Ud, oh)
        p.block_op_dev(which, Ud, op_)
        torch.cuda.synchronize()
        ref = _block_ref(o, U, h.g, ss, which)
        assert _rel(oh.cpu().numpy(), op_.cpu().numpy()) <= 1e-13, which
        assert _rel(oh.cpu().numpy(), ref) <= TOL, (which, _rel(oh.cpu().numpy(), ref))
    # single-mode applies on a harmonic handle keep the per-mode caches
    q = gaussian_charge(xy)
    for m in (0, 2 * ks - 2):
        assert _rel(h.mapping(q, m), o.mapping(q, m)) <= TOL


@pytest.mark.parametrize("sz,d,ks", [(16, 1, 5), (11, 3, 2)])
def test_harmonic_symmetric_blocks_match_directed(sz, d, ks, monkeypatch):
    """Stored-once V blocks read transposed by the partner (tau symmetric) against
    every directed block stored (ANISO_SYMMETRIC=0): same matvec to rounding."""
    torch = _torch()
    import aniso_amd

    outs = []
    for sym in ("1", "0"):
        monkeypatch.setenv("ANISO_SYMMETRIC", sym)
        a = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, 20)
        xy = a.getNodes()
        a.setCoeff(*rough_coeffs(xy, 6))
        for m in range(2 * ks - 1):
            a.cache(m)
        st = a.stats()
        assert st["harmonic"] == 1
        if sym == "1":
            assert st["att_m2l_blocks"] < st["m2l_pairs"]
        else:
            assert st["att_m2l_blocks"] == st["m2l_pairs"]
        U = torch.tensor(np.random.default_rng(1).uniform(-1, 1, (ks, a.N)), device="cuda")
        out = torch.zeros_like(U)
        a.block_op_dev(2, U, out)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    assert _rel(outs[0], outs[1]) <= 1e-13


@pytest.mark.parametrize("sz,d,ks,ml,sym,ring", [(32, 1, 5, 20, "1", "3x"), (19, 2, 3, 20, "1", "3x"),
                                                 (64, 1, 2, 20, "0", "3x"), (40, 1, 5, 3, "1", "3x"),
                                                 (32, 1, 5, 20, "1", "0"), (32, 1, 5, 20, "1", "2x"),
                                                 (32, 1, 5, 20, "1", "4x"), (24, 1, 8, 20, "1", "3x"),
                                                 (19, 2, 3, 20, "1", "0"), (32, 1, 5, 20, "1", "3v"),
                                                 (24, 1, 8, 20, "1", "3v"), (32, 1, 5, 20, "1", "3"),
                                                 (32, 1, 5, 20, "1", "0w4"), (32, 1, 5, 20, "1", "0w3"),
                                                 (64, 1, 2, 20, "0", "0w4"), (19, 2, 3, 20, "1", "0w4"),
                                                 (24, 1, 8, 20, "1", "0w4"), (32, 1, 5, 20, "1", "0w6"),
                                                 (32, 1, 5, 20, "1", "0h"), (19, 2, 3, 20, "1", "0h"),
                                                 (32, 1, 5, 20, "1", "3xh"), (24, 1, 8, 20, "1", "0h")])
def test_harmonic_clusters_match_per_target_waves(sz, d, ks, ml, sym, ring, monkeypatch):
    """The clustered harmonic M2L (in-cluster V pairs read once by
    the smaller id, both products, locals summed in LDS) against one wave per target
    (aniso_set_deterministic); odd sz (non-uniform tree), directed storage, a
    maxLevel-limited tree; the LDS-ring form at depths 2-4 with the target multipole
    in LDS (x) or VGPRs (v), every block count it compiles for (2, 4, 5, 8), the
    one-block-in-flight form (ANISO_HM_RING=0) and the default choice between them, that
    form at 4 waves per SIMD (w4: m2l_hc_cluster<LR>, <= 128 VGPRs; K = 8 keeps 3) and
    at 3 (w3: 4-wave workgroups; w6: 6-wave ones).  By default cross-cluster pairs are
    read once too (the halo form: partner products in LDS halo slots, folded into the
    locals after the launch); h: ANISO_HM_HALO=0, the directed copies instead.
    Also checks that in-cluster pairs exist, that the cluster plan reads fewer E
    blocks (the halo form: exactly the stored blocks), and that both deterministic
    forms (one wave per target; the clusters with fixed-point LDS sums, which take the
    one-block form whatever the ring knob says) repeat bitwise."""
    torch = _torch()
    import aniso_amd

    monkeypatch.setenv("ANISO_SYMMETRIC", sym)
    monkeypatch.setenv("ANISO_HM_RING", ring[0])
    if len(ring) > 1 and ring[1] in "xv":
        monkeypatch.setenv("ANISO_HM_RING_XL", "1" if ring[1] == "x" else "0")
    if "w" in ring:
        monkeypatch.setenv("ANISO_HM_WPE", ring[ring.index("w") + 1])
    halo = "h" not in ring
    monkeypatch.setenv("ANISO_HM_HALO", "1" if halo else "0")
    # 64-target clusters even at these sizes (the default depth keeps >= 512
    # clusters, which small trees only reach with 4-target clusters: no in-cluster pairs)
    monkeypatch.setenv("ANISO_HM_CLDEPTH", "3")
    outs, st = [], []
    for det in (False, True, "fixed"):
        monkeypatch.setenv("ANISO_DET_PER_TARGET", "0" if det == "fixed" else "1")
        a = aniso_amd.Aniso(sz, d, ks, 0.8, 8, 4, ml)
        a.set_deterministic(bool(det))
        xy = a.getNodes()
        a.setCoeff(*rough_coeffs(xy, 3))
        for m in range(2 * ks - 1):
            a.cache(m)
        st.append(a.stats())
        U = torch.tensor(np.random.default_rng(5).uniform(-1, 1, (ks, a.N)), device="cuda")
        out = torch.zeros_like(U)
        a.block_op_dev(2, U, out)
        if det:
            again = torch.zeros_like(U)
            a.block_op_dev(2, U, again)
            torch.cuda.synchronize()
            assert torch.equal(out, again)
        a.sync()
        outs.append(out.cpu().numpy())
    assert _rel(outs[2], outs[1]) <= 1e-13
    assert st[0]["harmonic"] == 1 and st[0]["hm_clusters"] > 0 and st[1]["hm_clusters"] == 0
    assert st[0]["hm_dual_pairs"] > 0 and st[0]["hm_block_reads"] < st[1]["hm_block_reads"]
    if not halo:
        assert st[0]["plan_halo_slots"] == 0
    if halo and sym == "1":  # every stored block read exactly once
        assert st[0]["hm_block_reads"] == st[0]["att_m2l_blocks"]
    assert _rel(outs[0], outs[1]) <= 1e-13


@pytest.mark.parametrize("ks,world,ring", [(5, 8, "3"), (2, 4, "3"), (3, 3, "3"), (5, 8, "0"), (5, 8, "0f"),
                                           (5, 8, "0w4"), (2, 4, "0fw4"), (5, 8, "0fw4")])
def test_small_clusters_on_shards_match_unsharded(ks, world, ring, monkeypatch):
    """The clustered M2L on the small clusters of an N-GPU shard (the adaptive depth
    gives 16-target clusters there) with 2, 4 (3 padded) and 5 blocks: every rank's
    two-phase apply equals the unsharded operator (the LDS-ring cluster form and the
    one-block-in-flight form; f: ANISO_TOP_FUSED=0, the upper tiers as launches of
    their own; w4: the one-block form at 4 waves per SIMD)."""
    torch = _torch()
    import aniso_amd

    monkeypatch.setenv("ANISO_HM_RING", ring[0])
    if "f" in ring:
        monkeypatch.setenv("ANISO_TOP_FUSED", "0")
    if "w4" in ring:
        monkeypatch.setenv("ANISO_HM_WPE", "4")
    sz = 256
    full = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 12)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(ks).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    full.block_op_dev(2, X, ref, tree=True)
    torch.cuda.synchronize()
    del full
    err, nans, _ = _two_phase_shards(sz, 1, ks, 20, coef, world, X, ref)
    assert nans == 0
    assert err <= 1e-13, err


@pytest.mark.parametrize("env", ["", "ANISO_DET_PER_TARGET=1", "ANISO_HM_HALO=0", "ANISO_HM_WPE=6"])
def test_deterministic_block_matvec_repeats_bitwise_at_config3_size(env, monkeypatch):
    """aniso_set_deterministic at BASELINE's 1M-point block matvec: repeat applies
    are bitwise identical, and equal the default (clustered) matvec to 1e-13.  The
    default runs the upper up tiers inside the M2L launch (k_top_m2l_hc), so this
    also checks its in-launch hand-offs against the plain tier launches.  Forms: the
    clustered M2L with fixed-point LDS sums (the default deterministic mode; with and
    without the halo slots, in 6-wave workgroups) and the round-2 per-target M2L."""
    torch = _torch()
    import aniso_amd

    for kv in filter(None, env.split(",")):
        k, v = kv.split("=")
        monkeypatch.setenv(k, v)
    a = aniso_amd.Aniso(1024, 1, 5, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*rough_coeffs(xy, 2))
    for m in range(9):
        a.cache(m)
    assert a.stats()["top_fused"] == 1
    U = torch.tensor(np.random.default_rng(8).uniform(-1, 1, (5, a.N)), device="cuda")
    ref = torch.zeros_like(U)
    a.block_op_dev(2, U, ref, tree=True)
    a.set_deterministic(True)
    o1, o2 = torch.zeros_like(U), torch.zeros_like(U)
    a.block_op_dev(2, U, o1, tree=True)
    a.block_op_dev(2, U, o2, tree=True)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert float(torch.linalg.norm(o1 - ref) / torch.linalg.norm(ref)) <= 1e-13


def test_deterministic_bounds_follow_a_new_shard_layout():
    """The fixed-point sums' per-cluster bounds are built from the plan (detBounds): a
    handle that ran deterministic applies on the whole tree and is then re-sharded
    must rebuild them, so its two-phase shard apply (with a second rank) still equals
    the default unsharded matvec and repeats bitwise."""
    torch = _torch()
    import aniso_amd

    sz, ks, world = 128, 5, 2
    full = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 4)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(3).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    full.block_op_dev(2, X, ref, tree=True)
    full.set_deterministic(True)
    tmp = torch.zeros_like(X)
    full.block_op_dev(2, X, tmp, tree=True)  # the whole tree's bounds
    torch.cuda.synchronize()
    hs = [full] + [aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20) for _ in range(world - 1)]
    for r, h in enumerate(hs):
        h.set_shard(r, world)
        h.setCoeff(*coef)
        for m in range(2 * ks - 1):
            h.cache(m)
        h.set_deterministic(True)
    got = []
    for rep in range(2):
        sends, outs, info = [], [], []
        for h in hs:
            b, e = h.shard()
            ex = h.shard_exchange(ks)
            xr = torch.full_like(X, float("nan"))
            xr[:, b:e] = X[:, b:e]
            for lo, hi in h.shard_halo():
                xr[:, lo:hi] = X[:, lo:hi]
            y = torch.zeros(ks, max(e - b, 1), dtype=torch.float64, device="cuda")
            rs = torch.zeros(max(ex["root_chunk"] * ex["root_record"], 1), dtype=torch.float64, device="cuda")
            h.block_op_begin_dev(2, xr, y, rs)
            sends.append(rs[: ex["root_chunk"] * ex["root_record"]])
            outs.append(y)
            info.append((xr, b, e))
        recv = torch.cat(sends)
        Y = torch.zeros_like(X)
        for h, y, (xr, b, e) in zip(hs, outs, info):
            h.block_op_end_dev(2, xr, y, recv, world)
            Y[:, b:e] = y[:, : e - b]
        torch.cuda.synchronize()
        got.append(Y)
    assert torch.equal(got[0], got[1])
    assert not torch.isnan(got[0]).any()
    assert float(torch.linalg.norm(got[0] - ref) / torch.linalg.norm(ref)) <= 1e-13


@pytest.mark.parametrize("ks", [2, 4, 5, 8])
@pytest.mark.parametrize("scale", [1.0, 1e150, 1e-150])
def test_deterministic_fixed_point_sums_scale_and_block_counts(ks, scale):
    """The clustered M2L's fixed-point sums (harmonic.hip hc_det_scale) at every
    harmonic block count and at inputs 1e+-150 times the usual size (the cluster scale
    follows the multipoles; no overflow, no loss): bitwise repeats, and the default
    matvec's result to 1e-13.  A zero input gives zero."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(256, 1, ks, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*rough_coeffs(xy, 3))
    for m in range(2 * ks - 1):
        a.cache(m)
    U = scale * torch.tensor(np.random.default_rng(9).uniform(-1, 1, (ks, a.N)), device="cuda")
    ref = torch.zeros_like(U)
    a.block_op_dev(2, U, ref, tree=True)
    a.set_deterministic(True)
    o1, o2, z = torch.zeros_like(U), torch.zeros_like(U), torch.ones_like(U)
    a.block_op_dev(2, U, o1, tree=True)
    a.block_op_dev(2, U, o2, tree=True)
    a.block_op_dev(2, torch.zeros_like(U), z, tree=True)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.isfinite(o1).all()
    assert float(torch.linalg.norm(o1 - ref) / torch.linalg.norm(ref)) <= 1e-13
    assert not torch.any(z)


@pytest.mark.parametrize("knob", ["ANISO_OVERLAP=1", "ANISO_FUSE_SUB=0", "ANISO_HARMONIC=0", "ANISO_HM_RING=3",
                                  "ANISO_HM_WPE=3", "ANISO_HM_WPE=4", "ANISO_HM_WPE=6", "ANISO_HM_WPE=8",
                                  "ANISO_NEAR_IN_TOP=1,ANISO_OVERLAP=1", "ANISO_NEAR_WPE=3", "ANISO_TOP_FUSED=0",
                                  "ANISO_HM_HALO=0", "ANISO_NEAR_EARLY=0", "ANISO_NEAR_EARLY=0,ANISO_OVERLAP=1",
                                  "ANISO_NEAR_HS_SYM=1", "ANISO_NEAR_HS_SYM=1,ANISO_NEAR_EARLY=0",
                                  "ANISO_NEAR_HS_SYM=1,ANISO_OVERLAP=1", "ANISO_NEAR_HS_SYM=1,ANISO_TOP_FUSED=0",
                                  "ANISO_NEAR_ORDER=first,ANISO_OVERLAP=1", "ANISO_NEAR_UP=0", "ANISO_HM_TAIL=0",
                                  "ANISO_HM_TAIL=100000"])
def test_block_matvec_knobs_agree(knob, monkeypatch):
    """Every remaining environment knob of the block apply:
    the near field on a side stream beside the up pass and the M2L (one GPU's
    default is serial since round 5), the bottom up tier as its own launch instead of
    inside the near field (ANISO_NEAR_UP=0), the cluster M2L without its split tail
    clusters or with every regular cluster split (ANISO_HM_TAIL), the separate
    x - mforward(x) subtraction and the per-mode operator stream give the default's
    block matvec to rounding."""
    torch = _torch()
    import aniso_amd

    sz, ks = 32, 5
    outs = []
    for env in (None, knob):
        if env:
            for kv in env.split(","):
                k, v = kv.split("=")
                monkeypatch.setenv(k, v)
        a = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
        xy = a.getNodes()
        a.setCoeff(*rough_coeffs(xy, 4))
        for m in range(2 * ks - 1):
            a.cache(m)
        U = torch.tensor(np.random.default_rng(11).uniform(-1, 1, (ks, a.N)), device="cuda")
        out = torch.zeros_like(U)
        a.block_op_dev(2, U, out)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        a.close()
    assert _rel(outs[0], outs[1]) <= 1e-12


def _two_phase_shards(sz, d, ks, ml, coef, world, X, ref, g=0.8, ns=10):
    """Every rank's sharded apply in two phases, the root all-gather
    played by concatenating the ranks' send buffers: rank r's input holds X at its
    own range and halo and NaN everywhere else, so any read outside them poisons
    its output.  ks > 1: x - mforward(x) (aniso_block_op_*_dev, which = 2); ks = 1:
    main.cpp's forward operator (aniso_forward_tree_*_dev).  Returns (rel err of
    the assembled owned slices vs ref, NaN count, halo points / N)."""
    torch = _torch()
    import aniso_amd

    nb = X.shape[0]
    hs, outs, sends, halo = [], [], [], 0
    for r in range(world):
        sh = aniso_amd.Aniso(sz, d, ks, g, ns, 4, ml)
        sh.set_shard(r, world)
        sh.setCoeff(*coef)
        for m in range(2 * ks - 1):
            sh.cache(m)
        b, e = sh.shard()
        ex = sh.shard_exchange(nb)
        xr = torch.full_like(X, float("nan"))
        xr[:, b:e] = X[:, b:e]
        for lo, hi in sh.shard_halo():
            xr[:, lo:hi] = X[:, lo:hi]
            halo += hi - lo
        y = torch.zeros(nb, max(e - b, 1), dtype=torch.float64, device="cuda")
        rs = torch.zeros(max(ex["root_chunk"] * ex["root_record"], 1), dtype=torch.float64, device="cuda")
        if ks > 1:
            sh.block_op_begin_dev(2, xr, y, rs)
        else:
            sh.forward_tree_begin_dev(xr[0], y[0], rs)
        hs.append((sh, xr, (b, e), ex))
        outs.append(y)
        sends.append(rs[: ex["root_chunk"] * ex["root_record"]])
    recv = torch.cat(sends) if sends[0].numel() else torch.zeros(1, dtype=torch.float64, device="cuda")
    got = torch.zeros_like(X)
    for (sh, xr, (b, e), ex), y in zip(hs, outs):
        if ks > 1:
            sh.block_op_end_dev(2, xr, y, recv, world)
        else:
            sh.forward_tree_end_dev(xr[0], y[0], recv, world)
        got[:, b:e] = y[:, : e - b]
    torch.cuda.synchronize()
    nans = int(torch.isnan(got).sum())
    return float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref)), nans, halo / X.shape[1]


@pytest.mark.parametrize("sz,d,ks,ml,coeffs,world,sym", [
    (64, 1, 5, 20, "main", 2, 0), (64, 1, 5, 20, "rough", 8, 0), (48, 2, 3, 20, "rough", 3, 0),
    (30, 3, 1, 20, "main", 4, 0), (40, 1, 2, 3, "rough", 3, 0), (16, 1, 5, 20, "main", 3, 0),
    (11, 3, 1, 20, "rough", 2, 0), (1, 3, 1, 20, "main", 2, 0), (64, 1, 5, 20, "rough", 3, 1),
    (48, 2, 3, 20, "rough", 2, 1)])
def test_two_phase_sharded_apply_reads_only_own_and_halo(sz, d, ks, ml, coeffs, world, sym, monkeypatch):
    """The multi-GPU apply (own + halo up pass, tier-0 root all-gather, owned slice
    out) on NaN-poisoned inputs equals the unsharded tree-order operator: the
    exchange plan covers everything each rank's kernels read (uniform, odd-sized,
    maxLevel-limited and single-leaf trees; 1, 2, 3 (padded to 4) and 5 right-hand
    sides; even and odd world sizes; sym: the near field's symmetric U storage,
    whose pairs with a ghost leaf stay directed)."""
    torch = _torch()
    import aniso_amd

    if sym:
        monkeypatch.setenv("ANISO_NEAR_HS_SYM", "1")

    full = aniso_amd.Aniso(sz, d, ks, 0.8, 10, 4, ml)
    xy = full.getNodes()
    coef = main_coeffs(xy) if coeffs == "main" else rough_coeffs(xy, 3)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(sz).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    if ks > 1:
        full.block_op_dev(2, X, ref, tree=True)
    else:
        full.forward_tree_dev(X[0], ref[0])
    torch.cuda.synchronize()
    del full
    err, nans, _ = _two_phase_shards(sz, d, ks, ml, coef, world, X, ref)
    assert nans == 0
    assert err <= 1e-13, err


def test_block_matvec_eight_shards_at_config3_size():
    """The driver's 8-GPU bench path at full size, on one GPU: BASELINE's 1M-point
    block matvec (config 3) sharded by FMM subtree over 8 ranks -- each rank its own
    handle, input valid only at its own range and halo (NaN elsewhere), up pass over
    its own and halo subtrees, the tier-0 root multipoles exchanged, owned slice out
    -- equals the unsharded matvec."""
    torch = _torch()
    import aniso_amd

    sz, d, ks, g = 1024, 1, 5, 0.8
    full = aniso_amd.Aniso(sz, d, ks, g, 10, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 9)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    perm = torch.tensor(full.tree_perm(), device="cuda", dtype=torch.int64)
    U = torch.tensor(np.random.default_rng(11).uniform(-1, 1, (ks, full.N)), device="cuda")[:, perm].contiguous()
    ref = torch.zeros_like(U)
    full.block_op_dev(2, U, ref, tree=True)
    torch.cuda.synchronize()
    del full
    err, nans, halo = _two_phase_shards(sz, d, ks, 20, coef, 8, U, ref, g=g)
    assert nans == 0
    assert err <= 1e-13, err
    assert halo < 0.2  # halo points per rank / own points (1 ring of 16 x 16-point subtrees)


@pytest.mark.parametrize("sz", [256, 1024])
def test_config5_mixed_precision_16_rhs_matches_fp64_gmres(sz):
    """the config-3 geometry (sz = 1024 is the full 1M
    points), mode 0, 16 right-hand sides q_k (Gaussian bumps centred by
    mt19937_64(seed = k)), solved with an fp32 Krylov basis and the fp32 MFMA
    operator (fp32 caches, 16 right-hand sides per apply) in the inner solves and
    fp64 refinement over the fp64 batched device apply; each solution matches the
    fp64 single-RHS device GMRES (main.cpp:121-141) to 1e-10 (that GMRES is checked
    against the oracle's in test_config5_fp64_gmres_matches_oracle)."""
    torch = _torch()
    import aniso_amd
    from aniso_amd.solve import config5_charges, gmres_mixed, rhs_block

    a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    a.cache(0)
    k = 16
    Q = np.stack([config5_charges(xy, s) for s in range(k)])
    B = rhs_block(a, torch.tensor(Q, device="cuda"))
    X, outer, inner, rel = gmres_mixed(a, B, tol=1e-12, m=40, inner_tol=1e-6)
    torch.cuda.synchronize()
    assert (rel <= 1e-12).all() and outer >= 2
    Xh = X.cpu().numpy()
    for s in (0, 7, 15):  # fp64 reference solves (the C ABI's device GMRES)
        its, x, hist, fr = a.gmres(Q[s], m=80, maxit=400, tol=1e-12)
        assert its > 0
        assert _rel(Xh[s], x) <= 1e-10, (s, _rel(Xh[s], x))


def test_config5_library_solve_matches_torch_loop():
    """aniso_solve16_mixed_dev (config 5's whole solve in the library: fp64 refinement,
    fp32 inner GMRES on the DCGS2 Arnoldi of arnoldi16.hpp) against the torch-
    orchestrated loop it replaces (gmres_mixed(native=False), modified Gram-Schmidt):
    both reach 1e-12 in the same number of refinements and their solutions agree to
    1e-10; a zero right-hand side gives a zero column (no NaN from its zero residual);
    the restart length is checked."""
    torch = _torch()
    import aniso_amd
    from aniso_amd.solve import config5_charges, gmres_mixed, rhs_block

    a = aniso_amd.Aniso(256, 1, 1, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    a.cache(0)
    Q = np.stack([config5_charges(xy, s) for s in range(16)])
    B = rhs_block(a, torch.tensor(Q, device="cuda"))
    X1, o1, i1, r1 = gmres_mixed(a, B, tol=1e-12, m=40, inner_tol=1e-6)
    X0, o0, i0, r0 = gmres_mixed(a, B, tol=1e-12, m=40, inner_tol=1e-6, native=False)
    assert (r1 <= 1e-12).all() and o1 == o0 and o1 >= 2, (r1, o1, o0)
    assert abs(i1 - i0) <= max(2, i0 // 10), (i1, i0)
    for s in range(16):
        assert float(torch.linalg.norm(X1[s] - X0[s]) / torch.linalg.norm(X0[s])) <= 1e-10, s
    # a zero right-hand side (the torch loop's 0 / 0 residual would never converge)
    Bz = B.clone()
    Bz[5] = 0.0
    Xz, oz, iz, rz = gmres_mixed(a, Bz, tol=1e-12, m=40, inner_tol=1e-6)
    assert not torch.isnan(Xz).any() and (rz <= 1e-12).all() and rz[5] == 0.0
    assert float(torch.linalg.norm(Xz[5])) == 0.0
    for s in (0, 6, 15):
        assert float(torch.linalg.norm(Xz[s] - X1[s]) / torch.linalg.norm(X1[s])) <= 1e-10, s
    with pytest.raises(aniso_amd.AnisoError):
        a.solve16_mixed_dev(B, torch.zeros_like(B), m=48)


def test_config5_fp64_gmres_matches_oracle():
    """The fp64 reference solve of config 5 (the device GMRES, main.cpp:121-141) against
    the oracle's GMRES (gmres.cpp:53-169 restated) at sz = 256 (N = 65,536) for the
    first config-5 right-hand side: same iteration count, solutions within 1e-10."""
    _torch()
    import aniso_amd
    from aniso_amd.solve import config5_charges
    from oracle.oracle_py import Oracle

    sz = 256
    a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
    xy = a.getNodes()
    ss, st = main_coeffs(xy)
    a.setCoeff(ss, st)
    a.cache(0)
    q = config5_charges(xy, 0)
    j, x, hist, fr = a.gmres(q, m=80, maxit=400, tol=1e-12)
    o = Oracle(sz, 1, 1, 0.8, 10, 4, 20)
    o.setCoeff(ss, st)
    o.cache(0)
    jo, xo, ho, fro = o.gmres_main(q, 80, 400, 1e-12)
    o.close()
    assert j > 0 and jo == j, (j, jo)
    assert _rel(x, xo) <= 1e-10


def test_config2_full_size_matches_oracle():
    """BASELINE configs[1] at its full size (sz = 120, d = 3,
    ns = 8, maxLevel = 5, N = 129,600, ~127-point leaves): the device apply against the
    oracle for a random and a Gaussian charge (the oracle's cache takes ~20 s here)."""
    a, o, xy = _pair(120, 3, 1, 8, 5, "main")
    a.cache(0)
    o.cache(0)
    rng = np.random.default_rng(120)
    for q in (rng.uniform(-1, 1, a.N), gaussian_charge(xy)):
        assert _rel(a.mapping(q, 0), o.mapping(q, 0)) <= TOL


def test_config4_four_million_points_properties_and_shard():
    """BASELINE configs[3]'s geometry at full size (sz = 2048,
    d = 1, ns = 10, N = 4,194,304, mode 0): linearity, bitwise determinism and
    positivity of the device apply, and one rank of its 8-way subtree sharding
    reproducing the owned slice of the unsharded tree-order forward operator."""
    torch = _torch()
    import aniso_amd

    sz = 2048
    a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
    assert a.N == 4 * 1024 * 1024
    xy = a.getNodes()
    coef = main_coeffs(xy)
    a.setCoeff(*coef)
    a.cache(0)
    rng = np.random.default_rng(4)
    q1 = torch.tensor(rng.uniform(-1, 1, a.N), device="cuda")
    q2 = torch.tensor(gaussian_charge(xy), device="cuda")
    o1, o2, o3, o4 = (torch.zeros_like(q1) for _ in range(4))
    a.mapping_dev(q1, 0, o1)
    a.mapping_dev(q2, 0, o2)
    a.mapping_dev(2.5 * q1 - 0.75 * q2, 0, o3)
    a.mapping_dev(q1, 0, o4)
    torch.cuda.synchronize()
    lin = 2.5 * o1 - 0.75 * o2
    assert float(torch.linalg.norm(o3 - lin) / torch.linalg.norm(lin)) <= 1e-13
    assert torch.equal(o1, o4)
    assert float(o2.min()) > 0
    perm = torch.tensor(a.tree_perm(), device="cuda", dtype=torch.int64)
    xt = q1[perm].contiguous()
    full = torch.zeros_like(xt)
    a.forward_tree_dev(xt, full)
    torch.cuda.synchronize()
    del a
    r, world = 5, 8
    sh = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
    sh.set_shard(r, world)
    sh.setCoeff(*coef)
    sh.cache(0)
    b, e = sh.shard()
    part = torch.zeros(e - b, dtype=torch.float64, device="cuda")
    sh.forward_tree_dev(xt, part)
    torch.cuda.synchronize()
    ref = full[b:e]
    assert float(torch.linalg.norm(part - ref) / torch.linalg.norm(ref)) <= 1e-14


@pytest.mark.parametrize("sz,d,ml,coeffs", [(64, 1, 20, "main"), (30, 3, 20, "rough"), (24, 1, 2, "rough"),
                                            (11, 3, 20, "main"), (13, 2, 20, "rough"), (1, 3, 20, "main")])
def test_fp32_mfma_operator_matches_fp64(sz, d, ml, coeffs):
    """Config 5's fp32 operator (16 right-hand sides, every FMM translation on
    v_mfma_f32_16x16x4_f32, fp32 caches) against the fp64 forward operator
    (main.cpp:125-136) column by column: fp32 agreement (<= 2e-6 relative, the
    inner solver's operator; the outer refinement keeps the fp64 one).  Uniform,
    d = 3 (9-point squares), maxLevel-limited (36-point leaves), odd sz, and the
    single-leaf tree."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(sz, d, 1, 0.8, 8, 4, ml)
    xy = a.getNodes()
    a.setCoeff(*(main_coeffs(xy) if coeffs == "main" else rough_coeffs(xy, 5)))
    a.cache(0)
    rng = np.random.default_rng(sz + d)
    X = torch.tensor(rng.uniform(-1, 1, (a.N, 16)), device="cuda", dtype=torch.float32)
    Y = torch.zeros_like(X)
    a.forward_f32_dev(X, Y)
    Xd = X.double().t().contiguous()
    ref = torch.zeros_like(Xd)
    for j in range(16):
        a.forward_tree_dev(Xd[j], ref[j])
    torch.cuda.synchronize()
    err = float(torch.linalg.norm(Y.double().t() - ref) / torch.linalg.norm(ref))
    # the operator part alone (X - Y vs X - ref): fp32 relative accuracy of K_0
    kerr = float(torch.linalg.norm((Xd - Y.double().t()) - (Xd - ref)) / torch.linalg.norm(Xd - ref))
    assert err <= 2e-6 and kerr <= 2e-5, (err, kerr)


@pytest.mark.parametrize("ks", [2, 3, 5])
def test_fused_top_of_tree_launch_matches_tier_launches(ks):
    """The block operator's upper up tiers inside the clustered M2L launch
    (k_top_m2l_hc: in-launch per-tier counters, waiting clusters) against the
    bitwise-deterministic path, which runs every tier as a launch of its own, for
    every compiled right-hand-side count the harmonic path uses (2, 4 = 3 padded, 5)."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(256, 1, ks, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*rough_coeffs(xy, 6))
    for m in range(2 * ks - 1):
        a.cache(m)
    assert a.stats()["top_fused"] == 1
    U = torch.tensor(np.random.default_rng(9).uniform(-1, 1, (ks, a.N)), device="cuda")
    outs = []
    for det in (False, True, False):
        a.set_deterministic(det)
        out = torch.zeros_like(U)
        a.block_op_dev(2, U, out)
        a.sync()  # raises if an in-launch hand-off timed out (its output would be invalid)
        outs.append(out.cpu().numpy())
    assert _rel(outs[0], outs[1]) <= 1e-13 and _rel(outs[2], outs[1]) <= 1e-13


def test_stage_timer_levels():
    """aniso_set_timing: level 1 times every stage, level 2 (bench.py's timed region)
    only the M2L and near-field spans; the output is the same at every level, and a
    level outside 0..2 is ANISO_ERR_INVALID."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(128, 1, 5, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*rough_coeffs(xy, 6))
    for m in range(9):
        a.cache(m)
    U = torch.tensor(np.random.default_rng(4).uniform(-1, 1, (5, a.N)), device="cuda")
    outs, times = [], []
    for level in (0, 1, 2):
        a.set_timing(level)
        out = torch.zeros_like(U)
        for _ in range(2):
            a.block_op_dev(2, U, out)
        a.sync()
        times.append(a.stage_times())
        a.set_timing(0)
        outs.append(out.cpu().numpy())
    assert _rel(outs[1], outs[0]) <= 1e-13 and _rel(outs[2], outs[0]) <= 1e-13
    full, roof = times[1], times[2]
    assert all(full[k] > 0 for k in ("up", "m2l", "near", "down", "total"))
    assert roof["m2l"] > 0 and roof["near"] > 0
    assert all(roof[k] == 0 for k in ("exchange", "up", "gather", "down", "corr", "total"))
    with pytest.raises(aniso_amd.AnisoError):
        a.set_timing(3)


@pytest.mark.parametrize("nv", [1, 7, 16, 17, 40, 60])
def test_krylov_primitives_match_torch(nv):
    """aniso_krylov_dot / _update (the CGS2 sweeps of the block solve and of
    gmres_dist: register-held bases up to 48 vectors, the two-pass kernels above)
    against torch fp64 on random bases, n not a multiple of the block size."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(8, 1, 2, 0.8, 10, 4, 20)
    g = torch.Generator(device="cuda").manual_seed(nv)
    n = 300_007
    V = torch.rand(nv, n, dtype=torch.float64, device="cuda", generator=g) - 0.5
    w = torch.rand(n, dtype=torch.float64, device="cuda", generator=g) - 0.5
    c = torch.rand(nv, dtype=torch.float64, device="cuda", generator=g) - 0.5
    out = torch.zeros(nv + 1, dtype=torch.float64, device="cuda")
    a.krylov_dot(V, w, out)
    ref = V @ w
    assert float((out[:nv] - ref).abs().max() / ref.abs().max()) <= 1e-12
    w1, w2 = w.clone(), w.clone()
    a.krylov_update(V, c, w1, out, dots=True)
    wr = w - V.t() @ c
    assert float((w1 - wr).abs().max() / wr.abs().max()) <= 1e-12
    assert float((out[:nv] - V @ wr).abs().max() / (V @ wr).abs().max()) <= 1e-12
    assert abs(float(out[nv]) - float(wr @ wr)) <= 1e-12 * float(wr @ wr)
    sq = torch.zeros(1, dtype=torch.float64, device="cuda")
    a.krylov_update(V, c, w2, sq, dots=False)
    assert torch.equal(w1, w2)
    assert abs(float(sq[0]) - float(wr @ wr)) <= 1e-12 * float(wr @ wr)


def test_gmres_dist_on_library_sweeps_matches_torch_path():
    """gmres_dist with kry (the library's sweeps, device scaling, the next matvec ahead
    of the rotations) takes the same steps as its torch path on the block operator
    and lands on the same solution."""
    torch = _torch()
    import aniso_amd
    from aniso_amd.solve import gmres_dist

    a = aniso_amd.Aniso(32, 1, 5, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    for m in range(9):
        a.cache(m)
    b = torch.tensor(np.random.default_rng(3).uniform(-1, 1, (5, a.N)), device="cuda")

    def apply(x, y):
        a.block_op_dev(2, x, y, tree=True)

    for restart in (6, 40):
        h0, h1 = [], []
        x0, its0, r0 = gmres_dist(apply, b, restart=restart, tol=1e-11, maxit=20, hist=h0)
        x1, its1, r1 = gmres_dist(apply, b, restart=restart, tol=1e-11, maxit=20, hist=h1, kry=a)
        assert its0 == its1 and its1 > 0 and r1 <= 1e-11
        assert np.allclose(h0, h1, rtol=1e-6, atol=1e-14)
        assert float(torch.linalg.norm(x1 - x0) / torch.linalg.norm(x0)) <= 1e-10


def test_loopback_communicator_runs_a_rank_schedule():
    """aniso_comm_init_loopback (development: one rank's schedule of an N-GPU run on
    one GPU, tools/shard_time.py --native): the one-call sharded matvec runs on it and
    leaves finite values in the owned slice (the other ranks' roots are left out, so
    they are not the operator's)."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(64, 1, 5, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.set_shard(1, 4)
    a.setCoeff(*rough_coeffs(xy, 6))
    for m in range(9):
        a.cache(m)
    a.comm_init_loopback()
    b, e = a.shard()
    X = torch.tensor(np.random.default_rng(4).uniform(-1, 1, (5, a.N)), device="cuda")
    Y = torch.full_like(X, float("nan"))
    a.block_op_sharded_dev(2, X, Y)
    a.sync()
    assert bool(torch.isfinite(Y[:, b:e]).all())


def test_fused_launch_timeline(monkeypatch):
    """ANISO_TOP_TRACE=1 (development): aniso_top_trace returns one record per block of
    the last fused top-of-tree launch -- the up tasks of tiers 1.. first, then every
    cluster once -- with start <= end of wait <= end on the 100 MHz clock."""
    torch = _torch()
    import aniso_amd

    monkeypatch.setenv("ANISO_TOP_TRACE", "1")
    a = aniso_amd.Aniso(128, 1, 5, 0.8, 10, 4, 20)
    xy = a.getNodes()
    a.setCoeff(*rough_coeffs(xy, 4))
    for m in range(9):
        a.cache(m)
    assert a.stats()["top_fused"] == 1
    U = torch.tensor(np.random.default_rng(2).uniform(-1, 1, (5, a.N)), device="cuda")
    out = torch.zeros_like(U)
    a.block_op_dev(2, U, out, tree=True)
    tr = a.top_trace()
    st = a.stats()
    assert tr.shape[1] == 8 and tr.shape[0] > st["hm_clusters"] > 0
    up = tr[tr[:, 4] < 0]
    cl = tr[tr[:, 4] >= 0]
    assert len(cl) == st["hm_clusters"] and sorted(cl[:, 4].tolist()) == list(range(st["hm_clusters"]))
    assert (np.diff(-up[:, 4]) >= 0).all()  # tiers in order
    assert (tr[:, 0] <= tr[:, 1]).all() and (tr[:, 1] <= tr[:, 2]).all() and (tr[:, 0] > 0).all()
    assert int(cl[:, 7].sum()) == st["hm_block_reads"]


def test_fused_top_of_tree_waits_compute_what_they_wait_for(monkeypatch):
    """A hand-off wait of k_top_m2l_hc that polls its tier counter ANISO_TOP_SPIN_LIMIT
    times without seeing the tier complete computes the tier's tasks itself (after the
    tiers below), so no wait can hang on, or be spoiled by, a producer block that is not
    resident (no dispatch-order assumption).  Forced here at once (limit 0: every
    waiting block computes every tier it reads): the host-pointer block operator, the
    device-pointer one followed by aniso_sync, and aniso.m's block solve all return the
    default handle's results, no time-out is reported, and aniso_stats counts the tasks
    the waiters computed (top_steals)."""
    torch = _torch()
    import aniso_amd

    monkeypatch.setenv("ANISO_TOP_SPIN_LIMIT", "0")
    ks = 5
    a = aniso_amd.Aniso(256, 1, ks, 0.8, 10, 4, 20)
    monkeypatch.delenv("ANISO_TOP_SPIN_LIMIT")
    xy = a.getNodes()
    a.setCoeff(*main_coeffs(xy))
    for m in range(2 * ks - 1):
        a.cache(m)
    assert a.stats()["top_fused"] == 1
    b = aniso_amd.Aniso(256, 1, ks, 0.8, 10, 4, 20)
    b.setCoeff(*main_coeffs(xy))
    for m in range(2 * ks - 1):
        b.cache(m)
    Uh = np.random.default_rng(1).uniform(-1, 1, (ks, a.N))
    ref = b.block_op(2, Uh)
    got = a.block_op(2, Uh)
    st = a.stats()
    assert st["top_recoveries"] == 0 and st["top_fused"] == 1 and st["top_steals"] > 0
    assert _rel(got, ref) <= 1e-13
    U = torch.tensor(Uh, device="cuda")
    out = torch.zeros_like(U)
    a.block_op_dev(2, U, out)
    a.sync()  # nothing to report
    assert _rel(out.cpu().numpy(), ref) <= 1e-13
    # aniso.m's solve (aniso.m:159-173)
    rhs = np.zeros((ks, a.N))
    rhs[0] = np.exp(-25 * ((xy[:, 0] - 0.5) ** 2 + (xy[:, 1] - 0.5) ** 2))
    s0 = a.stats()["top_steals"]
    ita, xa, _, rela = a.block_solve(rhs.reshape(-1), restart=20, tol=1e-10, maxit=10)
    itb, xb, _, relb = b.block_solve(rhs.reshape(-1), restart=20, tol=1e-10, maxit=10)
    assert ita == itb > 0 and rela <= 1e-10
    assert a.stats()["top_steals"] > s0 and b.stats()["top_steals"] == 0 and b.stats()["top_recoveries"] == 0
    assert _rel(xa, xb) <= 1e-9


def test_set_coeff_rebuilds_fp32_caches():
    """Config 5's fp32 operator after a second setCoeff + cache(0) runs on the new
    sigma_t's caches (they are rounded from the mode-0 operators), and before that
    cache(0) it fails as a state error instead of using the old ones."""
    torch = _torch()
    import aniso_amd

    a = aniso_amd.Aniso(64, 1, 1, 0.8, 10, 4, 20)
    xy = a.getNodes()
    X = torch.tensor(np.random.default_rng(2).uniform(-1, 1, (a.N, 16)), device="cuda", dtype=torch.float32)
    Y = torch.zeros_like(X)
    a.setCoeff(*main_coeffs(xy))
    a.cache(0)
    a.forward_f32_dev(X, Y)
    a.setCoeff(*rough_coeffs(xy, 8))
    with pytest.raises(aniso_amd.AnisoError) as ei:
        a.forward_f32_dev(X, Y)
    assert ei.value.code == 3
    a.cache(0)
    a.forward_f32_dev(X, Y)
    Xd = X.double().t().contiguous()
    ref = torch.zeros_like(Xd)
    for j in range(16):
        a.forward_tree_dev(Xd[j], ref[j])
    torch.cuda.synchronize()
    err = float(torch.linalg.norm(Y.double().t() - ref) / torch.linalg.norm(ref))
    assert err <= 2e-6, err


def test_sharded_end_must_repeat_its_begin():
    """Phase 2 of a sharded apply checks that it repeats its phase 1 (operation, which,
    vectors, strides): a mismatched _end is a state error and leaves the begun apply
    pending, and the matching _end then completes it correctly."""
    torch = _torch()
    import aniso_amd

    sz, ks, world = 32, 5, 2
    full = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
    xy = full.getNodes()
    coef = main_coeffs(xy)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(4).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    full.block_op_dev(2, X, ref, tree=True)
    hs = []
    for r in range(world):
        sh = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
        sh.set_shard(r, world)
        sh.setCoeff(*coef)
        for m in range(2 * ks - 1):
            sh.cache(m)
        ex = sh.shard_exchange(ks)
        rs = torch.zeros(max(ex["root_chunk"] * ex["root_record"], 1), dtype=torch.float64, device="cuda")
        y = torch.zeros(ks, sh.n_owned(), dtype=torch.float64, device="cuda")
        sh.block_op_begin_dev(2, X, y, rs)
        hs.append((sh, y, rs[: ex["root_chunk"] * ex["root_record"]]))
    recv = torch.cat([h[2] for h in hs])
    sh, y, _ = hs[0]
    y2 = torch.zeros_like(y)
    for bad in (lambda: sh.block_op_end_dev(1, X, y, recv, world), lambda: sh.block_op_end_dev(2, X, y2, recv, world),
                lambda: sh.forward_tree_end_dev(X[0], y[0], recv, world)):
        with pytest.raises(aniso_amd.AnisoError) as ei:
            bad()
        assert ei.value.code == 3
    got = []
    for sh, y, _ in hs:
        sh.block_op_end_dev(2, X, y, recv, world)
        got.append(y)
    torch.cuda.synchronize()
    got = torch.cat(got, 1)
    assert float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref)) <= 1e-13


def _block_ref_per_mode(o, U, g, ss):
    """x - mforward(x) (aniso.m:138-157, 155) composed from oracle mode applies, the
    oracle holding one mode's caches at a time (its 9-mode cache would not fit at
    full size): for every mode m, each input block b the mixes use is applied once."""
    import aniso_amd

    nb = U.shape[0]
    mix = aniso_amd.block_mixes(nb, g, True)
    out = U.copy()
    for m in range(2 * nb - 1):
        o.cache(m)
        for b in range(nb):
            if np.any(mix[m, :, b]):
                y = o.mapping(U[b] * ss, m)
                for i in range(nb):
                    if mix[m, i, b]:
                        out[i] -= mix[m, i, b] * y
        o.uncache(m)
    return out


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_config3_full_size_odd_mode_matches_oracle():
    """BASELINE's headline geometry at its FULL size (config 3: sz = 1024, d = 1,
    ns = 10, N = 1,048,576) against the oracle apply (AnisoWrapper.cpp:92-136
    restated) for an odd mode (m = 5) with varying sigma: <= 1e-10 relative.  The
    oracle's one-mode cache takes ~40 s on the box's cores."""
    a, o, xy = _pair(1024, 1, 5, 10, 20, "main")
    m = 5
    a.cache(m)
    o.cache(m)
    q = gaussian_charge(xy) + np.random.default_rng(1024).uniform(-0.1, 0.1, a.N)
    err = _rel(a.mapping(q, m), o.mapping(q, m))
    o.close()
    assert err <= TOL, err


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_block_matvec_sz512_matches_oracle_composition():
    """aniso.m's GMRES matvec x - mforward(x) on the harmonic block path (all 9 modes x
    5 blocks in one apply, the bench's operator) at sz = 512 (N = 262,144) against the
    oracle's per-mode composition (45 mapping calls in aniso.m's loop): <= 1e-10."""
    torch = _torch()
    a, o, xy = _pair(512, 1, 5, 10, 20, "main")
    ks, ss = 5, main_coeffs(xy)[0]
    for m in range(2 * ks - 1):
        a.cache(m)
    assert a.stats()["harmonic"] == 1
    U = np.random.default_rng(512).uniform(-1, 1, (ks, a.N))
    U[0] += gaussian_charge(xy)
    Ud = torch.tensor(U, device="cuda")
    out = torch.zeros_like(Ud)
    a.block_op_dev(2, Ud, out)
    a.sync()
    got = out.cpu().numpy()
    ref = _block_ref_per_mode(o, U, a.g, ss)
    o.close()
    assert _rel(got, ref) <= TOL, _rel(got, ref)


def _gmres_matlab(apply, b, restart, tol, maxit):
    """Restarted GMRES with MATLAB's stopping rule (relative residual <= tol, checked
    per step on the estimate and confirmed explicitly at each cycle's end), modified
    Gram-Schmidt, numpy on the host: the reference solve of aniso.m:159-173 over the
    oracle's operator.  Returns (x, total steps, final relative residual)."""
    x = np.zeros_like(b)
    nb = np.linalg.norm(b)
    r = b - apply(x)
    beta = np.linalg.norm(r)
    total = 0
    for _ in range(maxit):
        if beta / nb <= tol:
            break
        V = np.zeros((restart + 1, b.size))
        H = np.zeros((restart + 1, restart))
        V[0] = r / beta
        g = np.zeros(restart + 1)
        g[0] = beta
        cs, sn = np.zeros(restart), np.zeros(restart)
        used = 0
        for i in range(restart):
            w = apply(V[i])
            for k in range(i + 1):
                H[k, i] = V[k] @ w
                w = w - H[k, i] * V[k]
            H[i + 1, i] = np.linalg.norm(w)
            V[i + 1] = w / H[i + 1, i]
            for k in range(i):
                t = cs[k] * H[k, i] + sn[k] * H[k + 1, i]
                H[k + 1, i] = -sn[k] * H[k, i] + cs[k] * H[k + 1, i]
                H[k, i] = t
            den = np.hypot(H[i, i], H[i + 1, i])
            cs[i], sn[i] = H[i, i] / den, H[i + 1, i] / den
            H[i, i], H[i + 1, i] = den, 0.0
            g[i + 1], g[i] = -sn[i] * g[i], cs[i] * g[i]
            total += 1
            used = i + 1
            if abs(g[i + 1]) / nb <= tol:
                break
        y = np.linalg.solve(np.triu(H[:used, :used]), g[:used])
        x = x + V[:used].T @ y
        r = b - apply(x)
        beta = np.linalg.norm(r)
    return x, total, beta / nb


@pytest.mark.parametrize("sz,restart", [(32, 400), (48, 8)])
def test_block_solve_matches_gmres_over_oracle(sz, restart):
    """aniso.m:159-173's solve -- rhs = forward(charge), u = gmres(A, rhs, restart,
    1e-11, 400) with A(u) = u - mforward(u) -- through aniso_block_solve (every Krylov
    vector in HBM, CGS2 on the device) against the same restarted GMRES over the
    oracle's 45-call composition (a host MGS restatement with MATLAB's stopping rule)
    and SciPy's gmres: the same step count as the restatement, solutions within 1e-10,
    with a restart short enough to cycle (restart 8) and MATLAB's 400."""
    from scipy.sparse.linalg import LinearOperator, gmres

    _torch()
    a, o, xy = _pair(sz, 1, 5, 10, 20, "main")
    ks, ss = 5, main_coeffs(xy)[0]
    for m in range(2 * ks - 1):
        a.cache(m)
        o.cache(m)
    charge = np.zeros((ks, a.N))
    charge[0] = gaussian_charge(xy)  # demo.m:24-29: the source in block 0
    rhs = _block_ref(o, charge, a.g, ss, 0).reshape(-1)

    def A(v):
        return _block_ref(o, np.asarray(v, dtype=np.float64).reshape(ks, a.N), a.g, ss, 2).reshape(-1)

    tol = 1e-11
    xr, its_ref, rr_ref = _gmres_matlab(A, rhs, restart, tol, 400)
    its, u, hist, rr = a.block_solve(rhs, restart, tol, 400)
    assert its > 0 and rr <= tol and rr_ref <= tol
    assert its == its_ref, (its, its_ref)
    assert _rel(u.reshape(-1), xr) <= 1e-10, _rel(u.reshape(-1), xr)
    assert hist.size == its and hist[-1] <= tol
    xs, info = gmres(LinearOperator((rhs.size, rhs.size), matvec=A, dtype=np.float64), rhs, rtol=tol,
                     restart=restart, maxiter=400)
    assert info == 0
    assert _rel(u.reshape(-1), xs) <= 1e-10, _rel(u.reshape(-1), xs)
    # the device entry point on the same system, from a nonzero initial guess
    torch = _torch()
    rd = torch.tensor(rhs.reshape(ks, a.N), device="cuda")
    xd = torch.tensor(0.5 * xr.reshape(ks, a.N), device="cuda")
    its_d, _, rr_d = a.block_solve_dev(rd, xd, restart, tol, 400)
    assert its_d > 0 and rr_d <= tol
    assert _rel(xd.cpu().numpy().reshape(-1), xr) <= 1e-10


@pytest.mark.parametrize("sz,d,ml,coeffs", [(64, 1, 20, "main"), (30, 3, 20, "rough"), (24, 1, 2, "rough"),
                                            (11, 3, 20, "main"), (13, 2, 20, "rough"), (1, 3, 20, "main")])
def test_fp64_mfma_operator_matches_vector_path(sz, d, ml, coeffs):
    """The fp64 16-right-hand-side operator on v_mfma_f64_16x16x4_f64 (f64op.hip):
    main.cpp's forward operator and the mapping of modes 1 and 2 against the VALU
    path column by column (<= 1e-13: fp64 throughout, only the summation order
    differs), and aniso_mapping_batched for 11 and 16 columns (which runs on it)
    against per-column mapping and the oracle.  Uniform, d = 3, maxLevel-limited,
    odd sz, d = 2, and the single-leaf tree."""
    torch = _torch()
    a, o, xy = _pair(sz, d, 2, 8, ml, coeffs, seed=4)
    for m in range(3):
        a.cache(m)
    rng = np.random.default_rng(sz + d)
    X = torch.tensor(rng.uniform(-1, 1, (a.N, 16)), device="cuda")
    Y = torch.zeros_like(X)
    a.forward16_f64_dev(X, Y)
    Xc = X.t().contiguous()
    ref = torch.zeros_like(Xc)
    for j in range(16):
        a.forward_tree_dev(Xc[j], ref[j])
    torch.cuda.synchronize()
    assert float(torch.linalg.norm(Y.t() - ref) / torch.linalg.norm(ref)) <= 1e-13
    for m in (1, 2):
        a.mapping16_f64_dev(m, X, Y)
        for j in range(16):
            a.mapping_tree_dev(Xc[j], m, ref[j])
        torch.cuda.synchronize()
        assert float(torch.linalg.norm(Y.t() - ref) / torch.linalg.norm(ref)) <= 1e-13, m
    for k, m in ((11, 1), (16, 0)):
        Q = rng.uniform(-1, 1, (a.N, k))
        B = a.mapping_batched(Q, m)
        o.cache(m)
        for j in (0, k - 1):
            assert _rel(B[:, j], a.mapping(Q[:, j], m)) <= 1e-13
            assert _rel(B[:, j], o.mapping(Q[:, j], m)) <= TOL



def test_native_exchange_one_rank_rccl_and_callbacks():
    """The library's own exchange (aniso_comm_init_rccl / _callbacks +
    aniso_block_op_sharded_dev: halo all-to-all, phase 1, root all-gather, phase 2 in
    one call) on a one-rank shard: RCCL itself (a one-rank communicator; RCCL refuses
    two ranks on one GPU) and caller-supplied callbacks equal the unsharded operator."""
    torch = _torch()
    import aniso_amd

    ks = 5
    full = aniso_amd.Aniso(64, 1, ks, 0.8, 10, 4, 20)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 2)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(6).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    full.block_op_dev(2, X, ref, tree=True)
    for kind in ("rccl", "callbacks"):
        sh = aniso_amd.Aniso(64, 1, ks, 0.8, 10, 4, 20)
        sh.set_shard(0, 1)
        sh.setCoeff(*coef)
        for m in range(2 * ks - 1):
            sh.cache(m)
        if kind == "rccl":
            sh.comm_init_rccl(aniso_amd.comm_unique_id())
        else:
            def ag(ctx, send, recv, count, stream):
                aniso_amd.memcpy(recv, send, 8 * count)
                return 0

            def a2a(ctx, send, sc, so, recv, rc, ro, stream):
                return 0 if sc[0] == 0 and rc[0] == 0 else 1

            def ar(ctx, buf, count, stream):
                return 0

            sh.comm_init_callbacks(aniso_amd.Collectives(None, aniso_amd.COLL_ALLGATHER(ag),
                                                         aniso_amd.COLL_ALLTOALLV(a2a), aniso_amd.COLL_ALLREDUCE(ar)))
        y = torch.zeros_like(X)
        sh.block_op_sharded_dev(2, X.clone(), y)
        sh.sync()
        assert float(torch.linalg.norm(y - ref) / torch.linalg.norm(ref)) <= 1e-13, kind


class _ThreadCollectives:
    """aniso_collectives between handles of one process, one thread per rank (the
    ranks share the box's one GPU; ctypes drops the GIL inside the library's calls):
    host-staged through shared slots and a barrier."""

    def __init__(self, world, rank, shared):
        import aniso_amd

        self.world, self.rank, self.sh, self.lib = world, rank, shared, aniso_amd
        self.struct = aniso_amd.Collectives(None, aniso_amd.COLL_ALLGATHER(self._ag),
                                            aniso_amd.COLL_ALLTOALLV(self._a2a), aniso_amd.COLL_ALLREDUCE(self._ar))

    def _host(self, ptr, n):
        buf = np.empty(int(n), dtype=np.float64)
        if n:
            self.lib.memcpy(buf.ctypes.data, ptr, 8 * int(n))
        return buf

    def _put(self, ptr, arr):
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if arr.size:
            self.lib.memcpy(ptr, arr.ctypes.data, 8 * arr.size)

    def _guard(self, fn):
        try:
            fn()
            return 0
        except Exception as ex:  # noqa: BLE001 -- the library turns the status into its error
            self.sh["errors"].append(repr(ex))
            self.sh["bar"].abort()
            return 1

    def _ag(self, ctx, send, recv, count, stream):
        def run():
            self.sh["slot"][self.rank] = self._host(send, count)
            self.sh["bar"].wait()
            self._put(recv, np.concatenate([self.sh["slot"][r] for r in range(self.world)]))
            self.sh["bar"].wait()
        return self._guard(run)

    def _a2a(self, ctx, send, sc, so, recv, rc, ro, stream):
        def run():
            self.sh["slot"][self.rank] = [self._host(send + 8 * int(so[p]), int(sc[p])) for p in range(self.world)]
            self.sh["bar"].wait()
            for p in range(self.world):
                if p != self.rank and int(rc[p]):
                    part = self.sh["slot"][p][self.rank]
                    assert part.size == int(rc[p])
                    self._put(recv + 8 * int(ro[p]), part)
            self.sh["bar"].wait()
        return self._guard(run)

    def _ar(self, ctx, buf, count, stream):
        def run():
            self.sh["slot"][self.rank] = self._host(buf, count)
            self.sh["bar"].wait()
            self._put(buf, np.sum([self.sh["slot"][r] for r in range(self.world)], axis=0))
            self.sh["bar"].wait()
        return self._guard(run)


@pytest.mark.parametrize("sz,world,one,d,ml", [(64, 2, "1", 1, 20), (64, 2, "0", 1, 20), (64, 4, "1", 1, 20),
                                               (64, 8, "1", 1, 20), (64, 3, "1", 1, 20), (96, 3, "1", 1, 20),
                                               (40, 2, "1", 1, 3), (32, 2, "1", 2, 20), (64, 3, "mixed", 1, 20),
                                               (64, 2, "spin0", 1, 20), (256, 4, "1", 1, 20), (512, 8, "1", 1, 20),
                                               (256, 4, "partial0", 1, 20), (512, 8, "tails", 1, 20),
                                               (256, 4, "det", 1, 20)])
def test_native_exchange_ranks_as_threads(sz, world, one, d, ml, monkeypatch):
    """The library's one-call sharded block matvec (aniso_block_op_sharded_dev) with
    `world` ranks as threads of one process on the box's GPU, each rank's input valid
    only at its own range (NaN elsewhere), the collectives host-staged between the
    threads: the one-collective exchange (own tier-0 subtrees, then the roots, the
    multipoles below the root level and the input the rank reads from each owner in
    one grouped exchange) and, with ANISO_ONE_EXCHANGE=0 or where the cuts split a
    tier-0 subtree, the two-collective one; the owned slices equal the unsharded
    matvec.  The maxLevel-limited tree (leaves above 16 points: no staged near field)
    and d = 2 (no fused corrections) take the two-collective form by themselves.
    "mixed": rank 0's process would allow the one-collective form and the others' not
    (ANISO_ONE_EXCHANGE differs per handle): the ranks must still agree (ADVICE r04:
    the decision is all-gathered at comm_init), here on the two-collective form.
    "spin0": ANISO_TOP_SPIN_LIMIT=0, every waiting block of the fused launch computes
    the upper tiers it reads (the sharded phase 2, from the gathered roots; with
    ANISO_UPPER_PARTIAL=0, since the partial sums leave phase 2 no up tier).
    The one-collective form exchanges the upper multipoles as partial sums where every
    rank's plan forms them (records at 256 and 512 points per side; "partial0":
    ANISO_UPPER_PARTIAL=0, the root records and the upper tiers on every rank).
    "det": every rank in the deterministic mode (fixed-point cluster sums): the two
    matvecs are bitwise equal on every rank, and equal the default unsharded one."""
    torch = _torch()
    import threading

    import aniso_amd

    monkeypatch.setenv("ANISO_ONE_EXCHANGE", "1" if one in ("mixed", "spin0", "partial0", "tails", "det") else one)
    # "tails": the upper partial tasks as tails of the own tier-0 launch (ANISO_UP_TAILS=1)
    monkeypatch.setenv("ANISO_UP_TAILS", "1" if one == "tails" else "0")
    monkeypatch.setenv("ANISO_UPPER_PARTIAL", "0" if one in ("spin0", "partial0") else "1")
    ks = 5
    full = aniso_amd.Aniso(sz, d, ks, 0.8, 10, 4, ml)
    xy = full.getNodes()
    coef = rough_coeffs(xy, 2)
    full.setCoeff(*coef)
    for m in range(2 * ks - 1):
        full.cache(m)
    X = torch.tensor(np.random.default_rng(world).uniform(-1, 1, (ks, full.N)), device="cuda")
    ref = torch.zeros_like(X)
    full.block_op_dev(2, X, ref, tree=True)
    torch.cuda.synchronize()
    hs = []
    for r in range(world):
        if one == "mixed":
            monkeypatch.setenv("ANISO_ONE_EXCHANGE", "1" if r == 0 else "0")
        if one == "spin0":  # every waiting block of the fused launch computes its tiers (no hand-off)
            monkeypatch.setenv("ANISO_TOP_SPIN_LIMIT", "0")
        h = aniso_amd.Aniso(sz, d, ks, 0.8, 10, 4, ml)
        h.set_shard(r, world)
        h.setCoeff(*coef)
        for m in range(2 * ks - 1):
            h.cache(m)
        h.set_deterministic(one == "det")
        hs.append(h)
    oks = [h.shard_exchange_one()["ok"] for h in hs]
    staged = d == 1 and ml == 20  # the harmonic near field from the input, fused corrections
    shared = dict(bar=threading.Barrier(world, timeout=60), slot=[None] * world, errors=[])
    colls = [_ThreadCollectives(world, r, shared) for r in range(world)]
    outs = [None] * world

    def run(r):
        try:
            h = hs[r]
            h.comm_init_callbacks(colls[r].struct)
            b, e = h.shard()
            x = torch.full_like(X, float("nan"))
            x[:, b:e] = X[:, b:e]
            y = torch.zeros_like(X)
            first = None
            for _ in range(2):  # a second matvec reuses the exchange plan
                h.block_op_sharded_dev(2, x, y)
                if first is None:
                    first = y[:, b:e].clone()
            h.sync()
            outs[r] = y[:, b:e].clone()
            if one == "det" and not torch.equal(first, outs[r]):
                raise AssertionError(f"rank {r}: deterministic matvecs differ")
        except Exception as ex:  # noqa: BLE001
            shared["errors"].append(repr(ex))
            shared["bar"].abort()

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not shared["errors"], shared["errors"]
    Y = torch.cat(outs, dim=1)
    assert not torch.isnan(Y).any()
    assert float(torch.linalg.norm(Y - ref) / torch.linalg.norm(ref)) <= 1e-13
    used = [h.stats()["one_exchange_applies"] for h in hs]
    one_used = one in ("1", "spin0", "partial0", "tails", "det") and all(oks) and staged
    assert used == [2 * int(one_used)] * world
    ups = [h.shard_upper_partials() for h in hs]
    assert [h.stats()["upper_partial_applies"] for h in hs] == [2 * int(one_used and all(u["on"] for u in ups))] * world
    if sz >= 256 and one == "1":
        assert all(u["on"] and u["records"] > 0 for u in ups)
    if one == "spin0":
        assert all(h.stats()["top_steals"] > 0 for h in hs)


@pytest.mark.parametrize("world,uncached", [(2, 1), (3, 0)])
def test_comm_init_fails_on_every_rank_when_one_rank_is_uncached(world, uncached):
    """A rank that has not cached its modes cannot run its part of a sharded matvec;
    the ranks learn it together: comm_init all-gathers every rank's cache readiness
    and fails on EVERY rank (no rank is left waiting inside a collective), and a
    sharded matvec without a communicator is an error as well."""
    _torch()
    import threading

    import aniso_amd

    ks, sz = 3, 32
    hs = []
    for r in range(world):
        h = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
        h.set_shard(r, world)
        h.setCoeff(*rough_coeffs(h.getNodes(), 2))
        if r != uncached:
            for m in range(2 * ks - 1):
                h.cache(m)
        hs.append(h)
    shared = dict(bar=threading.Barrier(world, timeout=60), slot=[None] * world, errors=[])
    colls = [_ThreadCollectives(world, r, shared) for r in range(world)]
    codes = [None] * world

    def run(r):
        try:
            hs[r].comm_init_callbacks(colls[r].struct)
            codes[r] = 0
        except aniso_amd.AnisoError as ex:
            codes[r] = ex.code

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(60)
    assert not any(t.is_alive() for t in threads)
    assert not shared["errors"], shared["errors"]
    assert all(c not in (None, 0) for c in codes), codes
    import torch

    x = torch.zeros(ks, hs[0].N, dtype=torch.float64, device="cuda")
    with pytest.raises(aniso_amd.AnisoError):
        hs[0].block_op_sharded_dev(2, x, torch.zeros_like(x))
