#!/usr/bin/env python3
"""bench.py -- GMRES matvec throughput of the MI355X path at 1M quadrature points.

Workload (BASELINE.json metric "GMRES matvec/s & pair-interactions/s at 1M quad
points"): the configs[2] geometry (sz=1024, d=1, ns=10, np=4, maxLevel=20,
N = 1,048,576), main.cpp's coefficient functions, and main.cpp's GMRES matvec
forwardOperator u - K_0(sigma_s .* u) (main.cpp:125-136): one apply of mode 0 per
matvec.  A "step" is one matvec; steps are chained (v <- A v) with every vector
resident in HBM, kept in tree order (a fixed relabelling of the unknowns, so no
permutation gathers on the data path).  fp64 throughout.

N GPUs (torchrun, one process per GPU, RCCL): the target set is sharded by FMM
subtree (strong scaling: total work fixed).  Each rank applies its shard; one
all-gather of tree-ordered slices rebuilds the replicated output vector.

Also reported on the same JSON line:
  roofline      HBM roofline of the dominant kernel (k_m2l), timed with HIP events
                on the apply stream over the timed region;
  cpu_baseline  the CPU oracle (a faithful port of the reference apply) on this
                host's cores, on a bounded sample of the same geometry family;
  rel_err_vs_cpu  GPU vs CPU oracle on that sample's inputs.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy


def main_coeffs(xy):
    """main.cpp:34-40"""
    x = xy[:, 0]
    ss = 16 * 0.5 * (1 - np.cos(2 * np.pi * x))
    return ss, ss + 0.2


def gaussian(xy):
    """main.cpp:29-32"""
    return np.exp(-25 * ((xy[:, 0] - 0.5) ** 2 + (xy[:, 1] - 0.5) ** 2))


def ref_pairs(sz, d, ns, s):
    """Reference pair interactions per apply: 2 P_U + 2 P_M + P_rem + P_R + P_S."""
    N = sz * sz * d * d
    p_rem = d ** 4 * (3 * sz - 2) ** 2
    p_r = 16 * d ** 4 * ((3 * sz - 2) ** 2 - sz ** 2)
    p_s = 8 * ns * ns * N
    return 2 * s["near_entries"] + 2 * s["m2l_entries"] + p_rem + p_r + p_s


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/rNN_pmc_summary.json, made by tools/profile_round.sh + tools/pmc_summary.py
    on this same bench command; FETCH_SIZE doubled per the gfx950 correction)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not files:
        return None, None
    k = json.load(open(files[-1]))["kernels"].get(kernel)
    if not k:
        return None, None
    return int(k["traffic_bytes"]), os.path.relpath(files[-1], ROOT)


def cpu_baseline(args, gpu_check):
    """Oracle (oracle/, a faithful CPU port of the reference apply incl. the per-apply
    tree rebuild) on a bounded sample; returns (baseline dict, rel err vs GPU)."""
    from oracle.oracle_py import Oracle

    sz = args.cpu_sz
    o = Oracle(sz, args.d, 1, 0.8, args.ns, 4, args.max_level)
    xy = o.getNodes()
    ss, st = main_coeffs(xy)
    o.setCoeff(ss, st)
    t0 = time.time()
    o.cache(0)
    t_cache = time.time() - t0
    q = gaussian(xy)
    u = q * ss
    o.mapping(u, 0)  # warm-up
    reps, t0 = 0, time.time()
    while reps < 3 or time.time() - t0 < args.cpu_seconds:
        ref = o.mapping(u, 0)
        reps += 1
    t_apply = (time.time() - t0) / reps
    rel = gpu_check(sz, u, ref)
    scale = float(args.sz * args.sz) / float(sz * sz)  # O(N) extrapolation to the workload
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {
        "value": 1.0 / (t_apply * scale),
        "unit": "matvec/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle apply (mode 0, tree rebuilt per apply as in the reference) at sz={sz} "
                   f"(N={sz * sz * args.d ** 2}) of the same d={args.d}, ns={args.ns} geometry, {reps} reps, "
                   f"{t_apply * 1e3:.1f} ms/apply, extrapolated linearly in N to N={args.sz * args.sz * args.d ** 2}; "
                   f"cache build {t_cache:.1f} s not timed; OMP threads={cores}"),
    }, rel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sz", type=int, default=1024)
    ap.add_argument("--d", type=int, default=1)
    ap.add_argument("--ns", type=int, default=10)
    ap.add_argument("--max-level", type=int, default=20)
    ap.add_argument("--cpu-sz", type=int, default=512, help="CPU baseline sample size (sz; N = sz^2 d^2)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline timing budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N>1 (gloo = CPU-staged rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on cuda:0 (rehearse the sharded path on a one-GPU box; use --backend gloo)")
    ap.add_argument("--verify", action="store_true", help="check the sharded matvec against an unsharded operator")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import aniso_amd
    from aniso_amd import dist as adist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = 0 if args.same_device else local
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    op = aniso_amd.Aniso(args.sz, args.d, 5, 0.8, args.ns, 4, args.max_level)
    N = op.N
    xy = op.getNodes()
    ss, st = main_coeffs(xy)
    full_stats = op.stats()
    perm = torch.tensor(op.tree_perm(), device="cuda", dtype=torch.int64)
    if world > 1:
        ranges = adist.shard_ranges(op, world)
        op.set_shard(rank, world)
        L = adist.pad_len(ranges)
        slice_buf = torch.zeros(L, dtype=torch.float64, device="cuda")
        gathered = torch.zeros(world, L, dtype=torch.float64, device="cuda")
        gidx = torch.tensor(adist.gather_index(ranges, L), device="cuda")
        b_own, e_own = ranges[rank]
    op.setCoeff(ss, st)
    t0 = time.time()
    op.cache(0)
    torch.cuda.synchronize()
    t_cache = time.time() - t0
    # GMRES vectors live in tree order (a fixed relabelling of the unknowns): the
    # forward operator then needs no permutation gathers, and the shards' output
    # slices concatenate to the next iterate
    v = torch.tensor(gaussian(xy), device="cuda")[perm].contiguous()
    w = torch.zeros_like(v)

    def matvec(x, y):
        if world == 1:
            op.forward_tree_dev(x, y)
            return
        op.forward_tree_dev(x, slice_buf)  # writes the owned e_own - b_own entries
        if args.backend == "nccl":
            dist.all_gather_into_tensor(gathered, slice_buf)
        else:  # gloo rehearsal: stage through host memory
            parts = [torch.zeros(L, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, slice_buf.cpu())
            gathered.copy_(torch.stack(parts))
        torch.index_select(gathered.view(-1), 0, gidx, out=y)

    for _ in range(args.warmup):
        matvec(v, w)
        v, w = w, v
    op.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        matvec(v, w)
        v, w = w, v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    times = op.stage_times()  # per-apply averages over the timed region (HIP events)
    op.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    my_stats = op.stats()
    ms = 1e3 * elapsed / args.steps
    value = args.steps / elapsed
    # dominant kernel: k_m2l (streams the stored merged 16x16 M2L operators once:
    # 2 KB per stored block, + multipole read and local write per target node, +
    # one 128-B transposed partial per canonical pair)
    m2l_bytes = (2048.0 * my_stats["stored_m2l"] + 2.0 * 128.0 * my_stats["m2l_targets"]
                 + 128.0 * my_stats["m2l_canon"])
    m2l_ms = times["m2l"]
    achieved = m2l_bytes / (m2l_ms * 1e-3) / 1e9 if m2l_ms > 0 else 0.0
    traffic, tsrc = pmc_traffic("aniso::k_m2l") if world == 1 and args.sz == 1024 and args.d == 1 else (None, None)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "k_m2l",
                "kernel_ms": round(m2l_ms, 5), "algorithmic_bytes": int(m2l_bytes), "traffic_source": tsrc}
    line = {
        "metric": "GMRES matvec/s at 1M quadrature points (main.cpp forwardOperator, mode 0)",
        "value": round(value, 3),
        "unit": "matvec/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: main.cpp coefficient functions and Gaussian source on the unit square",
        "config": {"workload": "configs[2] geometry (1M points, d=1, ns=10, np=4, maxLevel=20), GMRES matvec of mode 0",
                   "N": N, "sz": args.sz, "d": args.d, "ns": args.ns, "np": 4, "maxLevel": args.max_level,
                   "parallelism": f"fmm-subtree-shard x{world}" if world > 1 else "single-gpu"},
        "pair_interactions_per_s": round(value * ref_pairs(args.sz, args.d, args.ns, full_stats), 1),
        "stage_ms": {k: round(v_, 5) for k, v_ in times.items()},
        "cache_build_s": round(t_cache, 3),
        "roofline": roofline,
    }
    if args.verify:
        # one matvec of a fixed vector through this (possibly sharded) path vs an
        # unsharded operator on the same device
        u = torch.tensor(gaussian(xy), device="cuda")
        got = torch.zeros_like(u)
        matvec(u[perm].contiguous(), got)  # tree order in and out
        ref_op = aniso_amd.Aniso(args.sz, args.d, 5, 0.8, args.ns, 4, args.max_level)
        ref_op.setCoeff(ss, st)
        ref_op.cache(0)
        ref = torch.zeros_like(u)
        ref_op.forward_dev(u, ref)  # original order, unsharded
        torch.cuda.synchronize()
        ref = ref[perm]
        line["verify_rel_err_vs_unsharded"] = float(torch.linalg.norm(got - ref) / torch.linalg.norm(ref))
        del ref_op
    if rank == 0 and world == 1 and not args.no_cpu:
        def gpu_check(sz, u, ref):
            a = aniso_amd.Aniso(sz, args.d, 1, 0.8, args.ns, 4, args.max_level)
            a.setCoeff(*main_coeffs(a.getNodes()))
            a.cache(0)
            got = a.mapping(u, 0)
            return float(np.linalg.norm(got - ref) / np.linalg.norm(ref))

        base, rel = cpu_baseline(args, gpu_check)
        line["cpu_baseline"] = base
        line["rel_err_vs_cpu"] = rel
        line["speedup_vs_cpu"] = round(value / base["value"], 1)
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
