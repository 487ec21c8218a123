#!/usr/bin/env python3
"""Extract the reference's Gauss-Legendre tables as a golden DATA fixture.

The reference hard-codes its 1-D Gauss-Legendre rules as decimal literals in
`get_legendre_data` (/root/reference/Quadrature.cpp:5418-22191).  The node order
is NOT sorted (e.g. degree 3 is 0, -0.77, +0.77; Quadrature.cpp:5430-5437), and
the product and oracle must reproduce both the order and every bit.

This script reads that source file as TEXT, converts each literal with a correctly
rounded decimal->binary64 conversion (the same conversion a C++ compiler applies to
the literal), and writes `tests/golden/gauss_legendre_ref.json`:
    {"source": ..., "degrees": {"1": {"x": [...], "w": [...]}, ...}}
with every double stored as its float.hex() string.  Only numbers are stored (no
reference source text).  Run it in the survey container, where /root/reference
exists; the JSON is committed and travels to the GPU box instead of the reference.
"""
import json
import os
import re
import sys

REF = "/root/reference/Quadrature.cpp"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "gauss_legendre_ref.json")
MAX_DEG = 24  # keeps the fixture small; the build uses degrees 1..3 and 8..10


def main() -> int:
    text = open(REF).read()
    start = text.index("void get_legendre_data(size_t deg, Quadrature &table)")
    end = text.index("void affine(Quadrature &table)", start)
    body = text[start:end]
    blocks = re.split(r"deg == (\d+)\)", body)
    out = {}
    # blocks = [prefix, deg, block, deg, block, ...]
    for i in range(1, len(blocks), 2):
        deg = int(blocks[i])
        if deg > MAX_DEG:
            continue
        blk = blocks[i + 1]
        xs = {int(k): v for k, v in re.findall(r"points_x\[(\d+)\]\s*=\s*([-+0-9.eE]+)\s*;", blk)}
        ws = {int(k): v for k, v in re.findall(r"weights\[(\d+)\]\s*=\s*([-+0-9.eE]+)\s*;", blk)}
        assert len(xs) == deg and len(ws) == deg, (deg, len(xs), len(ws))
        out[str(deg)] = {
            "x": [float(xs[k]).hex() for k in range(deg)],
            "w": [float(ws[k]).hex() for k in range(deg)],
        }
    json.dump({"source": "Quadrature.cpp:get_legendre_data (values only, float.hex)",
               "degrees": out}, open(OUT, "w"), indent=0)
    print("wrote", OUT, "degrees", sorted(int(k) for k in out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
