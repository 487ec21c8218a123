"""Gauss-Legendre tables: generated header vs the reference's own table (golden fixture)."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _arr(h, name):
    s = h[h.index(name):]
    s = s[s.index("{") + 1 : s.index("};")]
    return [v.strip() for v in s.replace("\n", "").split(",") if v.strip()]


def test_generated_table_is_bit_exact_to_reference_fixture():
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "gauss_legendre_ref.json")))["degrees"]
    h = open(os.path.join(ROOT, "aniso_amd", "csrc", "gauss_legendre_table.h")).read()
    xs = [float.fromhex(v) for v in _arr(h, "aniso_gauss_x[]")]
    ws = [float.fromhex(v) for v in _arr(h, "aniso_gauss_w[]")]
    off = [int(v) for v in _arr(h, "aniso_gauss_off[]")]
    assert len(ref) >= 24
    for k, v in ref.items():
        n = int(k)
        o = off[n - 1]
        assert xs[o : o + n] == [float.fromhex(t) for t in v["x"]], n
        assert ws[o : o + n] == [float.fromhex(t) for t in v["w"]], n


def test_reference_order_is_unsorted_like_the_table():
    # Quadrature.cpp:5430-5437: degree 3 is 0, -x, +x
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "gauss_legendre_ref.json")))["degrees"]
    x3 = [float.fromhex(t) for t in ref["3"]["x"]]
    assert x3[0] == 0.0 and x3[1] < 0 < x3[2]
    for k, v in ref.items():
        w = [float.fromhex(t) for t in v["w"]]
        assert abs(sum(w) - 2.0) < 1e-13
