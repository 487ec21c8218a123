#!/usr/bin/env python3
"""Quick GPU bring-up check: HIP path vs oracle (small) and vs survey known answers.

Usage on the GPU box:  python tools/gpu_check.py [--big]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import aniso_amd  # noqa: E402
from oracle.oracle_py import Oracle  # noqa: E402


def coeffs(xy):
    x = xy[:, 0]
    ss = 16 * 0.5 * (1 - np.cos(2 * np.pi * x))
    return ss, ss + 0.2


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def small(sz, d, ks, ns, modes, seed=0):
    a = aniso_amd.Aniso(sz, d, ks, 0.8, ns, 4, 20)
    o = Oracle(sz, d, ks, 0.8, ns, 4, 20)
    xy = a.getNodes()
    assert np.array_equal(xy, o.getNodes())
    ss, st = coeffs(xy)
    a.setCoeff(ss, st)
    o.setCoeff(ss, st)
    rng = np.random.default_rng(seed)
    q = rng.uniform(-1, 1, a.N)
    import torch

    qd = torch.tensor(q, device="cuda")
    for m in modes:
        t0 = time.time()
        a.cache(m)
        t1 = time.time()
        o.cache(m)
        out = a.mapping(q, m)
        ref = o.mapping(q, m)
        st_ = o.mapping_stages(q, m)
        s = 1.0 / (2 * np.pi)
        stages = {
            "far+near": (aniso_amd.STAGE_FAR | aniso_amd.STAGE_NEAR, (st_[0] + st_[1]) * s),
            "stencil": (aniso_amd.STAGE_STENCIL, (st_[2] + st_[3]) * s),
            "sing": (aniso_amd.STAGE_SING, st_[4] * s),
        }
        res = {}
        for k, (mask, r) in stages.items():
            od = torch.zeros(a.N, dtype=torch.float64, device="cuda")
            a.mapping_dev(qd, m, od, mask=mask)
            torch.cuda.synchronize()
            res[k] = rel(od.cpu().numpy(), r)
        print(f"sz={sz} d={d} mode={m}: total rel {rel(out, ref):.3e}  stages {res}  gpu-cache {t1 - t0:.3f}s",
              flush=True)


def known(name):
    ka = json.load(open(os.path.join(ROOT, "tests", "golden", "survey_known_answers.json")))
    c = [x for x in ka["applies"] if x["name"] == name][0]
    t0 = time.time()
    a = aniso_amd.Aniso(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    t1 = time.time()
    xy = a.getNodes()
    ss, st = coeffs(xy)
    a.setCoeff(ss, st)
    t2 = time.time()
    a.cache(c["mode"])
    t3 = time.time()
    q = np.exp(-25 * ((xy[:, 0] - 0.5) ** 2 + (xy[:, 1] - 0.5) ** 2))
    out = a.mapping(q, c["mode"])
    t4 = time.time()
    n2 = float(np.sqrt(np.sum(out * out)))
    print(f"{name}: N={a.N} create {t1 - t0:.2f}s setCoeff {t2 - t1:.2f}s cache {t3 - t2:.2f}s apply(host) {t4 - t3:.3f}s")
    print(f"   norm {n2:.17e} ref {c['out_norm2']:.17e} rel {(n2 - c['out_norm2']) / c['out_norm2']:.3e}")
    print(f"   out0 rel {(out[0] - c['out0']) / c['out0']:.3e}  outHalf rel {(out[len(out) // 2] - c['outHalf']) / c['outHalf']:.3e}")
    import torch

    qd = torch.tensor(q, device="cuda")
    od = torch.zeros_like(qd)
    a.set_timing(True)
    a.mapping_dev(qd, c["mode"], od)
    torch.cuda.synchronize()
    print("   stage ms", a.stage_times(), a.stats(), flush=True)
    a.set_timing(False)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(10):
        a.mapping_dev(qd, c["mode"], od)
    torch.cuda.synchronize()
    print(f"   apply {1e3 * (time.time() - t0) / 10:.3f} ms", flush=True)


if __name__ == "__main__":
    print(aniso_amd.version(), flush=True)
    small(16, 3, 1, 8, [0])
    small(8, 1, 5, 10, range(9))
    small(12, 2, 2, 8, [0, 1, 2])
    known("probe256_d1")
    if "--big" in sys.argv:
        known("probe1M_d3")
