"""The N>1 path on CPU with gloo (world sizes 2 and 3): the host-side exchange plan
of the sharded apply (aniso_amd/dist.py) and the claim it rests on.

Every rank owns an FMM-subtree shard (a contiguous tree-order range).  Per apply it
runs the up pass only over the tier-0 subtrees its kernels read (own + halo), and
receives every other tier-0 root multipole through one all-gather; per iterate one
all-to-all refreshes its halo.  Here, per rank:

* the halo all-to-all (ShardExchange.halo over gloo) delivers exactly the owners'
  values at the rank's halo positions and touches nothing else;
* the root all-gather lands every rank's roots in the slots of aniso_shard_roots'
  receive map;
* the claim, checked with the CPU oracle (the reference algorithm): the rank's owned
  outputs depend on the input outside its own range and halo ONLY through the tier-0
  root multipoles.  A perturbation supported outside own + halo and in the null
  space of every skipped subtree's root P2M (bbfmm.h:737-748: S_x(i) S_y(j) w_p per
  point) leaves the owned outputs unchanged to rounding, while it does change other
  ranks' outputs.

The handle is host-only here (plans need no GPU); on the GPU box the same plan runs
the HIP apply over RCCL (bench.py, tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cheb_s(u, npc=4):
    """S(u, c_i) of bbfmm.h:653-655 for u in [-1, 1] (rows: points, columns: i)."""
    c = -np.cos((np.arange(npc) + 0.5) * np.pi / npc)
    Tu = np.stack([np.cos(l * np.arccos(np.clip(u, -1, 1))) for l in range(npc)], axis=1)
    Tc = np.stack([np.cos(l * np.arccos(c)) for l in range(npc)], axis=0)
    return (2.0 * Tu @ Tc - 1.0) / npc


def null_perturbation(op, rank_valid, rng):
    """delta (tree order): zero on the rank's valid positions and on the tier-0
    subtrees it runs; on every other tier-0 subtree a random vector in the null space
    of that root's P2M (16 x n_points: S_x(i) S_y(j) w_p)."""
    ints, geom = op.tree_nodes()
    ex = op.shard_exchange()
    L0 = ex["t0_level"]
    _, _, run = op.shard_roots()
    run = set(run.tolist())
    perm = op.tree_perm()
    xy = op.getNodes()
    w = op.getWeights()
    delta = np.zeros(op.N)
    skipped = 0
    for n in np.nonzero((ints[:, 5] == L0) & (ints[:, 8] == 0))[0]:
        if n in run:
            continue
        b, c = int(ints[n, 10]), int(ints[n, 9])
        pos = np.arange(b, b + c)
        assert not rank_valid[pos].any(), "a skipped subtree overlaps the rank's own range or halo"
        pts = perm[pos]
        cx, cy, rx, ry = geom[n]
        A = (cheb_s((xy[pts, 0] - cx) / rx)[:, None, :] * cheb_s((xy[pts, 1] - cy) / ry)[:, :, None]).reshape(c, 16)
        A = (A * w[pts, None]).T  # 16 x c
        d = rng.uniform(-1, 1, c)
        d -= A.T @ np.linalg.solve(A @ A.T, A @ d)
        delta[pos] = d
        skipped += 1
    return delta, skipped


def _worker(rank, world, port, result_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import aniso_amd
    from aniso_amd import dist as adist
    from oracle.oracle_py import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sz, d, ks, nb = 128, 1, 2, 2
        op = aniso_amd.Aniso(sz, d, ks, 0.5, 6, 4, 20)
        N = op.N
        op.set_shard(rank, world)
        x = adist.ShardExchange(op, rank, world, nb, "cpu", "gloo")
        b, e = x.own
        assert (b, e) == op.shard()
        valid = np.zeros(N, dtype=bool)
        valid[b:e] = True
        for lo, hi in x.halos[rank]:
            assert not valid[lo:hi].any(), "halo overlaps the own range"
            valid[lo:hi] = True
        # -- halo all-to-all: owners' values at the halo, nothing else touched
        y = torch.zeros(nb, N, dtype=torch.float64)
        ref = torch.arange(nb * N, dtype=torch.float64).reshape(nb, N) + 1.0
        y[:, b:e] = ref[:, b:e]
        x.halo(y)
        vm = torch.from_numpy(valid)
        halo_ok = bool(torch.equal(y[:, vm], ref[:, vm])) and bool((y[:, ~vm] == 0).all())
        # -- root all-gather: every rank's roots land in their receive slots
        send, recv, _ = op.shard_roots()
        rs = x.roots_send[: x.C * x.R].view(x.C, x.R)
        rs.zero_()
        rs[: len(send)] = torch.from_numpy(send.astype(np.float64))[:, None]
        x.roots_allgather()
        got = x.roots_recv[: world * x.C * x.R].view(world * x.C, x.R)
        slots = recv >= 0
        roots_ok = bool(torch.equal(got[torch.from_numpy(slots)][:, 0], torch.from_numpy(recv[slots].astype(np.float64))))
        roots_ok &= bool((got[torch.from_numpy(slots)] == got[torch.from_numpy(slots)][:, :1]).all())
        all_roots = set()
        for r in range(world):
            all_roots |= set(recv[r * x.C:(r + 1) * x.C][recv[r * x.C:(r + 1) * x.C] >= 0].tolist())
        roots_ok &= len(all_roots) == int(slots.sum())  # each root sent by exactly one rank
        # -- the claim, with the oracle: perturbations the rank never sees leave its outputs alone
        rng = np.random.default_rng(11 + rank)
        delta, skipped = null_perturbation(op, valid, rng)
        perm = op.tree_perm()
        o = Oracle(sz, d, ks, 0.5, 6, 4, 20)
        xy = o.getNodes()
        o.setCoeff(np.full(N, 2.0), 2.5 + np.sin(3 * xy[:, 0]))
        q = rng.uniform(-1, 1, N)
        dq = np.zeros(N)
        dq[perm] = delta
        errs, ctrl = [], []
        for m in (0, 1):
            o.cache(m)
            y0 = o.mapping(q, m)[perm]
            y1 = o.mapping(q + dq, m)[perm]
            o.uncache(m)
            errs.append(float(np.abs(y1[b:e] - y0[b:e]).max() / np.abs(y0[b:e]).max()))
            ctrl.append(float(np.abs(y1 - y0).max() / np.abs(y0).max()))
        o.close()
        result_q.put((rank, dict(halo_ok=halo_ok, roots_ok=roots_ok, skipped=skipped, errs=errs, ctrl=ctrl,
                                 halo_points=int(valid.sum() - (e - b)), own=e - b)))
    except Exception as ex:  # surface worker failures instead of hanging the queue
        result_q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_exchange_plan(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, v in res:
        assert isinstance(v, dict), v
        assert v["halo_ok"] and v["roots_ok"], (r, v)
        assert v["skipped"] > 0, (r, v)  # the test perturbs something
        assert max(v["errs"]) < 1e-12, (r, v)  # owned outputs: unchanged to rounding
        assert min(v["ctrl"]) > 1e-6, (r, v)  # ... while the perturbation is felt elsewhere
        assert v["halo_points"] < v["own"], (r, v)


def test_halo_plan_pairs_up():
    """send[r] of rank a == recv[a] of rank r, for a hand-made plan."""
    from aniso_amd import dist as adist

    cuts = [0, 10, 20, 30]
    halos = [[(10, 12)], [(8, 10), (20, 23)], [(15, 20), (29, 30)]]
    plans = [adist.halo_plan(cuts, halos, r) for r in range(3)]
    for a in range(3):
        for r in range(3):
            assert np.array_equal(plans[a][0][r], plans[r][1][a])
    assert plans[1][0][0].tolist() == [10, 11] and plans[1][0][2].tolist() == [15, 16, 17, 18, 19]



def _gmres_worker(rank, world, port, result_q):
    """gmres_dist over row shards of a dense stand-in operator (the call shape of the
    sharded block matvec: apply on this rank's slice, its own exchange inside), gloo
    all-reduces for the inner products."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from aniso_amd.solve import gmres_dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        A, b = _dense_problem()
        n = A.shape[0]
        cuts = [n * r // world for r in range(world + 1)]
        lo, hi = cuts[rank], cuts[rank + 1]
        Ar = A[lo:hi]

        def apply(x, y):  # all-gather the slices (the halo exchange's role), then the local rows
            parts = [torch.zeros(cuts[r + 1] - cuts[r], dtype=torch.float64) for r in range(world)]
            dist.all_gather(parts, x.contiguous())
            y.copy_(Ar @ torch.cat(parts))

        def allreduce(t):
            dist.all_reduce(t)
            return t

        hist = []
        x, its, rel = gmres_dist(apply, b[lo:hi].clone(), restart=12, tol=1e-11, maxit=20, allreduce=allreduce,
                                 hist=hist)
        result_q.put((rank, dict(x=x.numpy(), lo=lo, hi=hi, its=its, rel=rel, hist=hist)))
    except Exception as ex:
        result_q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


def _dense_problem():
    rng = np.random.default_rng(7)
    n = 240
    K = rng.uniform(-1, 1, (n, n)) / (2.3 * np.sqrt(n))
    A = torch.tensor(np.eye(n) - K)
    b = torch.tensor(rng.uniform(-1, 1, n))
    return A, b


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_gmres_matches_one_rank(world):
    """aniso_amd.solve.gmres_dist (CGS2: two all-reduces per Arnoldi step) over gloo
    row shards equals the one-rank solve: same step count (restarts included), the
    same residual history to rounding, the solution to 1e-10; and the one-rank solve
    equals the dense solution."""
    from aniso_amd.solve import gmres_dist

    A, b = _dense_problem()
    h1 = []
    x1, its1, rel1 = gmres_dist(lambda x, y: y.copy_(A @ x), b.clone(), restart=12, tol=1e-11, maxit=20, hist=h1)
    ref = np.linalg.solve(A.numpy(), b.numpy())
    assert its1 > 12 and rel1 <= 1e-11  # at least one restart
    assert np.linalg.norm(x1.numpy() - ref) / np.linalg.norm(ref) <= 1e-9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gmres_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = np.zeros(A.shape[0])
    for r in range(world):
        v = res[r]
        assert isinstance(v, dict), v
        assert v["its"] == its1, (v["its"], its1)
        assert np.allclose(v["hist"], h1, rtol=1e-6, atol=1e-14)
        x[v["lo"]:v["hi"]] = v["x"]
    assert np.linalg.norm(x - x1.numpy()) / np.linalg.norm(x1.numpy()) <= 1e-10


def _coll_worker(rank, world, port, result_q):
    """The host-staged callbacks of the library's exchange (aniso_amd.dist.HostCollectives),
    called through their C function pointers on host buffers (ctypes.memmove stands in
    for the device copies)."""
    import ctypes
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from aniso_amd.dist import HostCollectives

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = HostCollectives(world, copy=lambda d, s, n: ctypes.memmove(d, s, n))
        st = c.struct
        send = np.arange(3, dtype=np.float64) + 10 * rank
        recv = np.zeros(3 * world)
        rc1 = st.allgather(None, send.ctypes.data, recv.ctypes.data, 3, None)
        # alltoallv: rank r sends (r + 1) * (p + 1) values r * 100 + p to peer p != r
        sc = np.array([0 if p == rank else (rank + 1) * (p + 1) for p in range(world)], dtype=np.int64)
        so = np.concatenate([[0], np.cumsum(sc)[:-1]]).astype(np.int64)
        rcn = np.array([0 if p == rank else (p + 1) * (rank + 1) for p in range(world)], dtype=np.int64)
        ro = np.concatenate([[0], np.cumsum(rcn)[:-1]]).astype(np.int64)
        sbuf = np.concatenate([np.full(sc[p], rank * 100.0 + p) for p in range(world)])
        rbuf = np.zeros(int(rcn.sum()) + 1)
        P64 = ctypes.POINTER(ctypes.c_int64)
        rc2 = st.alltoallv(None, sbuf.ctypes.data, sc.ctypes.data_as(P64), so.ctypes.data_as(P64), rbuf.ctypes.data,
                           rcn.ctypes.data_as(P64), ro.ctypes.data_as(P64), None)
        red = np.array([1.0 + rank, 2.0 * rank])
        rc3 = st.allreduce(None, red.ctypes.data, 2, None)
        result_q.put((rank, dict(rc=(rc1, rc2, rc3), recv=recv, rbuf=rbuf[:-1], rcn=rcn, red=red, errors=c.errors)))
    except Exception as ex:
        result_q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_host_collectives_of_the_native_exchange(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_coll_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        v = res[r]
        assert isinstance(v, dict), v
        assert v["rc"] == (0, 0, 0) and not v["errors"], v
        assert np.array_equal(v["recv"], np.concatenate([np.arange(3) + 10 * p for p in range(world)]))
        want = np.concatenate([np.full(v["rcn"][p], p * 100.0 + r) for p in range(world)])
        assert np.array_equal(v["rbuf"], want)
        assert np.allclose(v["red"], [sum(1.0 + p for p in range(world)), sum(2.0 * p for p in range(world))])
