"""Pin the CPU oracle (oracle/) to the reference: tree/list/pair counts, apply and
GMRES known answers recorded by the survey's probe of the reference
(tests/golden/survey_known_answers.json; provenance inside)."""
import json
import os

import numpy as np
import pytest

from conftest import gaussian_charge, main_coeffs
from oracle.oracle_py import Oracle, OTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KA = json.load(open(os.path.join(ROOT, "tests", "golden", "survey_known_answers.json")))


def _counts(tr, np_=4):
    ni = tr.node_ints()
    U, V, W, X = (tr.lists(k) for k in range(4))
    empty = ni[:, 8].astype(bool)
    leaf = ni[:, 7].astype(bool)
    ns = ni[:, 9]
    near = m2l = 0
    nU = nV = nW = nX = 0
    for i in range(tr.nn):
        nV += int(sum(not empty[j] for j in V[i]))
        nX += int(sum(not empty[j] for j in X[i]))
        if leaf[i] and ns[i]:
            us = [j for j in U[i] if not empty[j]]
            ws = [j for j in W[i] if not empty[j]]
            nU += len(us)
            nW += len(ws)
            near += int(sum(ns[i] * ns[j] for j in us + ws))
    return dict(nodes=tr.nn, leaves=int(leaf.sum()), nearPairs=near, M2Lpairs=(nV + nX) * np_ ** 4,
                Ulist=nU, Vlist=nV, Wlist=nW, Xlist=nX, maxLevelUsed=tr.max_level, maxLeafPts=int(ns[leaf].max()))


@pytest.mark.parametrize("case", [t for t in KA["trees"] if t["N"] <= 1_100_000], ids=lambda t: t["name"])
def test_oracle_tree_matches_reference_counts(case):
    o = Oracle(case["sz"], case["d"], 1, 0.5, 8, case["np"], case["maxLevel"])
    xy = o.getNodes()
    tr = OTree(xy[:, 0], xy[:, 1], case["np"] ** 2, case["maxLevel"])
    got = _counts(tr, case["np"])
    for k, v in case.items():
        if k in got:
            assert got[k] == v, (case["name"], k, got[k], v)


def test_oracle_apply_matches_reference_known_answer():
    c = [a for a in KA["applies"] if a["name"] == "probe256_d1"][0]
    o = Oracle(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    xy = o.getNodes()
    ss, st = main_coeffs(xy)
    o.setCoeff(ss, st)
    o.cache(c["mode"])
    out = o.mapping(gaussian_charge(xy), c["mode"])
    assert abs(np.linalg.norm(out) - c["out_norm2"]) <= 1e-12 * c["out_norm2"]
    assert abs(out[0] - c["out0"]) <= 1e-11 * abs(c["out0"])
    assert abs(out[len(out) // 2] - c["outHalf"]) <= 1e-10 * abs(c["outHalf"])


@pytest.mark.slow
def test_oracle_gmres_matches_reference_iteration_count():
    c = KA["gmres"][0]
    o = Oracle(c["sz"], c["d"], c["ks"], c["g"], c["ns"], c["np"], c["maxLevel"])
    xy = o.getNodes()
    ss, st = main_coeffs(xy)
    o.setCoeff(ss, st)
    o.cache(0)
    j, x, hist, fr = o.gmres_main(gaussian_charge(xy), c["m"], c["maxit"], c["tol"])
    assert j == c["iterations"]
    assert hist[j - 1] == pytest.approx(c["final_resid_approx"], rel=0.1)  # printed "1.5e-12"
    assert fr < c["tol"]


def test_oracle_line_integral_is_partition_independent():
    """tau is the exact integral of a per-square polynomial: splitting a segment at
    any interior point must not change it (basis of the GPU DDA walk)."""
    o = Oracle(9, 3, 1, 0.5, 8, 4, 20)
    xy = o.getNodes()
    rng = np.random.default_rng(3)
    o.setCoeff(*(rng.uniform(0.5, 3.0, (2, o.N))))
    for _ in range(200):
        a, b = rng.uniform(0.01, 0.99, 2), rng.uniform(0.01, 0.99, 2)
        t = rng.uniform(0.05, 0.95)
        m = a + t * (b - a)
        whole = o.line_integral(a[0], a[1], b[0], b[1])
        parts = o.line_integral(a[0], a[1], m[0], m[1]) + o.line_integral(m[0], m[1], b[0], b[1])
        assert abs(whole - parts) <= 1e-12 * max(1.0, abs(whole))
