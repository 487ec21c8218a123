"""Host-side product logic on CPU: the C ABI library loads and exports every
symbol of include/aniso_mi355x.h; geometry and the quadtree / interaction lists
are bit-identical to the oracle's restatement of bbfmm::tree; argument / state
errors are reported like the reference's MEX errors; no CPU fallback exists."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import aniso_amd
from oracle.oracle_py import Oracle, OTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    names = aniso_amd.exported_symbols()
    assert len(names) >= 25
    # the drop-in boundary stays free of the development entries (aniso_mi355x_dev.h)
    public = aniso_amd.exported_symbols(public_only=True)
    for dev in ("aniso_top_trace", "aniso_comm_init_loopback", "aniso_line_integrals", "aniso_stage_times",
                "aniso_set_timing", "aniso_mapping_stages_dev", "aniso_tree_list"):
        assert dev in names and dev not in public, dev
    for core in ("aniso_create", "aniso_destroy", "aniso_num_nodes", "aniso_get_nodes", "aniso_set_coeff",
                 "aniso_cache", "aniso_mapping", "aniso_mapping_batched", "aniso_block_op", "aniso_block_solve"):
        assert core in public, core
    L = aniso_amd.lib()
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", aniso_amd.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}" in out, n
    assert "gfx950" in aniso_amd.version()


def test_library_contains_gfx950_code_object():
    blob = open(aniso_amd.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for k in (b"k_m2l", b"k_near", b"k_down_tier", b"k_up_tier", b"k_corr", b"k_cache_m2l"):
        assert k in blob, k


@pytest.mark.parametrize("sz,d,ns", [(1, 1, 8), (3, 2, 8), (16, 3, 8), (13, 3, 10)])
def test_geometry_matches_oracle_bit_exact(sz, d, ns):
    a = aniso_amd.Aniso(sz, d, 1, 0.5, ns, 4, 20)
    o = Oracle(sz, d, 1, 0.5, ns, 4, 20)
    assert a.N == o.N == sz * sz * d * d
    assert np.array_equal(a.getNodes(), o.getNodes())
    assert np.array_equal(a.getWeights(), o.weights())
    assert abs(a.getWeights().sum() - 1.0) < 1e-13


@pytest.mark.parametrize("sz,d,ml", [(1, 1, 20), (2, 1, 20), (16, 3, 20), (120, 3, 5), (7, 3, 20), (37, 2, 20),
                                     (50, 1, 3), (8, 2, 0), (97, 1, 20)])
def test_tree_and_lists_bit_exact_vs_oracle(sz, d, ml):
    a = aniso_amd.Aniso(sz, d, 1, 0.5, 8, 4, ml)
    xy = a.getNodes()
    ot = OTree(xy[:, 0], xy[:, 1], 16, ml)
    ints, geom = a.tree_nodes()
    oi, og = ot.node_ints(), ot.node_geom()
    assert ints.shape[0] == ot.nn
    assert np.array_equal(ints[:, :10], oi[:, :10])
    assert np.array_equal(geom, og)
    for w in range(4):
        ptr, idx = a.tree_list(w)
        ol = ot.lists(w)
        for i in range(ot.nn):
            assert np.array_equal(idx[ptr[i]:ptr[i + 1]], ol[i]), (w, i)
    perm = a.tree_perm()
    assert np.array_equal(np.sort(perm), np.arange(a.N))
    for i in range(ot.nn):
        if ints[i, 7]:  # leaves: same point order as the reference's sourceIndex
            assert np.array_equal(perm[ints[i, 10]:ints[i, 10] + ints[i, 9]], ot.sources(i))


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_shards_partition_targets_and_work(nranks):
    a = aniso_amd.Aniso(64, 1, 1, 0.5, 8, 4, 20)
    full = a.stats()
    ranges, leaves, near = [], 0, 0
    for r in range(nranks):
        a.set_shard(r, nranks)
        ranges.append(a.shard())
        s = a.stats()
        leaves += s["leaves"]
        near += s["near_entries"]
    assert ranges[0][0] == 0 and ranges[-1][1] == a.N
    for (b0, e0), (b1, e1) in zip(ranges, ranges[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in ranges]
    assert max(sizes) <= 1.6 * a.N / nranks
    assert leaves == full["leaves"] and near == full["near_entries"]


def test_errors_are_reported_not_swallowed():
    with pytest.raises(aniso_amd.AnisoError) as e:
        aniso_amd.Aniso(16, 3, 1, 0.5, 8, 5, 20)  # np must be 4
    assert e.value.code == 1
    with pytest.raises(aniso_amd.AnisoError):
        aniso_amd.Aniso(0, 3, 1, 0.5, 8, 4, 20)
    with pytest.raises(aniso_amd.AnisoError):
        aniso_amd.Aniso(4, 30, 1, 0.5, 8, 4, 20)  # quadrature degree not implemented
    a = aniso_amd.Aniso(4, 1, 2, 0.5, 8, 4, 20)
    with pytest.raises(aniso_amd.AnisoError) as e:
        a.cache(3)  # kernel ids 0..2
    assert e.value.code == 4
    with pytest.raises(aniso_amd.AnisoError) as e:
        a.cache(0)  # before setCoeff
    assert e.value.code == 3
    with pytest.raises(aniso_amd.AnisoError) as e:
        a.mapping(np.zeros(a.N), 0)  # before cache
    assert e.value.code == 3
    with pytest.raises(aniso_amd.AnisoError):
        a.mapping(np.zeros(a.N + 1), 0)
    L = aniso_amd.lib()
    assert L.aniso_cache(None, 0) == 5


def test_no_cpu_fallback_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    a = aniso_amd.Aniso(4, 1, 1, 0.5, 8, 4, 20)
    with pytest.raises(aniso_amd.AnisoError) as e:
        a.setCoeff(np.ones(a.N), np.ones(a.N))  # needs the HIP device
    assert e.value.code == 2


@pytest.mark.parametrize("nb,g", [(1, 0.8), (3, 0.5), (5, 0.8)])
def test_block_mixes_follow_aniso_m(nb, g):
    """aniso.m:121-157: output block iid gets chi_|j| K_{|iid+j|} u_|j| for every
    j in [-(nb-1), nb-1]; the mixes regroup those terms by mode."""
    for chi in (False, True):
        got = aniso_amd.block_mixes(nb, g, chi)
        ref = np.zeros((2 * nb - 1, nb, nb))
        for i in range(-(nb - 1), 1):
            iid = abs(i)
            for j in range(-(nb - 1), nb):
                b = abs(j)
                w = (g ** b - g ** nb) / (1 - g ** nb) if chi else 1.0
                ref[abs(i - j), iid, b] += w
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("env", ["1", "", "0"])
def test_block_near_symmetric_u_storage_plan(monkeypatch, env):
    """ANISO_NEAR_HS_SYM=1: block handles store a U pair of two owned leaves once
    (Plan::buildNearHs, the symmetric storage of bbfmm.h:1081-1099 applied to the
    harmonic near field): the stored E entries are the directed ones minus one
    direction of every such pair.  Off by default."""
    if env:
        monkeypatch.setenv("ANISO_NEAR_HS_SYM", env)
    a = aniso_amd.Aniso(64, 1, 5, 0.8, 8, 4, 20)
    s = a.stats()
    if env != "1":
        assert s["near_hs_stored"] == 0 and s["near_hs_partials"] == 0
        return
    ints, _ = a.tree_nodes()
    ptr, idx = a.tree_list(0)
    leaf = (ints[:, 7] == 1) & (ints[:, 8] == 0)
    cnt = ints[:, 9].astype(np.int64)
    skipped = 0
    for i in np.nonzero(leaf)[0]:
        for b in idx[ptr[i]:ptr[i + 1]]:
            if b > i and leaf[b]:
                skipped += cnt[i] * cnt[b]
    assert skipped > 0
    assert s["near_hs_stored"] == s["stored_near"] - skipped
    assert 0 < s["near_hs_partials"] < skipped
    # a shard keeps the pairs with a ghost leaf directed: every rank stores at least
    # its share, and the shards together store the directed entries of the cut pairs
    tot = 0
    for r in range(2):
        a.set_shard(r, 2)
        tot += a.stats()["near_hs_stored"]
    assert s["near_hs_stored"] < tot < s["stored_near"]


@pytest.mark.parametrize("sz,ks,nranks", [(64, 5, 2), (64, 5, 3), (64, 5, 8), (48, 2, 4)])
def test_one_collective_exchange_plan(sz, ks, nranks):
    """The one-collective exchange (Plan::buildExchange): each rank runs
    exactly the tier-0 tasks of its own subtrees (a partition of all of them), needs
    multipoles below the root level from other ranks, and reads fewer input points
    outside its range than the two-collective halo (its halo subtrees' points)."""
    a = aniso_amd.Aniso(sz, 1, ks, 0.8, 10, 4, 20)
    own_total, oks = 0, []
    for r in range(nranks):
        a.set_shard(r, nranks)
        one, two = a.shard_exchange_one(), a.shard_exchange(ks)
        assert one["own_t0_tasks"] == two["roots_sent"] <= two["t0_run"]
        own_total += one["own_t0_tasks"]
        oks.append(one["ok"])
        if one["ok"]:
            assert one["need_nodes"] > 0
            assert 0 < one["halo_points"] < two["halo_points"]
    assert own_total == a.shard_exchange(ks)["t0_tasks"]
    # at 3 ranks of 4,096 points the cuts split level-2 subtrees (the tier-0 roots):
    # those ranks keep the two-collective exchange (commInit requires every rank's ok)
    assert all(oks) == (nranks != 3)
    a.set_shard(0, 1)
    assert a.shard_exchange_one()["ok"] == 0  # one rank: nothing to exchange


@pytest.mark.parametrize("sz,nranks", [(256, 2), (256, 4), (512, 8), (128, 3)])
def test_upper_partial_sum_plan(sz, nranks, monkeypatch):
    """The upper multipoles as partial sums (Plan::xUpPartial): each rank's
    partial tasks cover exactly its own tier-0 roots, its records lie on the levels
    between the topmost one an M2L reads and the root level, and the ranks' records
    together reach every non-empty node there (each upper multipole is the sum of its
    records over the ranks).  Where the one-collective form is refused (3 ranks of 16,384
    points split tier-0 subtrees) or ANISO_UPPER_PARTIAL=0, no plan forms them."""
    a = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
    ints, _ = a.tree_nodes()
    level, empty = ints[:, 5], ints[:, 8]
    reached = set()
    ons = []
    for r in range(nranks):
        a.set_shard(r, nranks)
        one, u = a.shard_exchange_one(), a.shard_upper_partials()
        ons.append(u["on"])
        assert u["on"] == one["ok"]
        if not u["on"]:
            assert u["tasks"] == u["records"] == 0
            continue
        assert u["roots"] == one["own_t0_tasks"]
        lv = level[u["record_nodes"]]
        assert ((lv >= u["top_level"]) & (lv < u["root_level"])).all()
        reached.update(int(n) for n in u["record_nodes"])
    if all(ons):
        top, root = u["top_level"], u["root_level"]
        want = {n for n in range(len(level)) if top <= level[n] < root and not empty[n]}
        assert want and reached == want
    else:
        assert nranks == 3
    monkeypatch.setenv("ANISO_UPPER_PARTIAL", "0")
    b = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
    b.set_shard(0, nranks)
    assert b.shard_upper_partials()["on"] == 0


def test_bench_gpus_must_match_launcher_world_size():
    """bench.py --gpus N under a launcher whose WORLD_SIZE differs exits non-zero before
    touching torch or the GPU (the driver's N-GPU line must come from N ranks)."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode != 0
    assert "WORLD_SIZE=1" in out.stderr


def test_fixed_size_stats_writes_its_26_entries():
    """aniso_stats keeps the contract aniso_mi355x_dev.h gives it (26 entries, the same
    values aniso_stats_n reports first) and writes nothing past them."""
    a = aniso_amd.Aniso(16, 1, 3, 0.8, 10, 4, 20)
    full = np.zeros(40, dtype=np.int64)
    n = ctypes.c_int()
    P64 = ctypes.POINTER(ctypes.c_int64)
    assert aniso_amd.lib().aniso_stats_n(a.address, full.ctypes.data_as(P64), len(full), ctypes.byref(n)) == 0
    assert n.value == 34
    fixed = np.full(40, -7, dtype=np.int64)
    assert aniso_amd.lib().aniso_stats(a.address, fixed.ctypes.data_as(P64)) == 0
    assert np.array_equal(fixed[:26], full[:26])
    assert np.all(fixed[26:] == -7)
    a.close()
