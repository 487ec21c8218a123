"""Calibrate the CPU oracle (bench.py's cpu_baseline, kind "port") against the
reference's own recorded timings (SURVEY.md §6 / BASELINE.md: the survey's probe
build of the reference, OpenMP 8 threads on an 8-core Xeon VM, the class of host this
container is).  Times the oracle here with the same thread count on the same
geometries and prints one JSON line per case with the ratio oracle rate / reference
rate.  TEST INFRASTRUCTURE: loads oracle/ only.  usage: OMP_NUM_THREADS=8
python tools/calibrate_oracle.py [--refalloc]
(--refalloc: the oracle repeats the reference's per-use heap vectors and block copies,
oracle_set_reference_alloc; the results are unchanged)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import cpu_model, demo_coeffs, gaussian, main_coeffs  # noqa: E402
from oracle.oracle_py import Oracle  # noqa: E402

# (name, sz, d, ks, g, ns, maxLevel, coeffs, modes, reference applies/s, source)
CASES = [
    ("config1", 16, 3, 1, 0.0, 8, 20, main_coeffs, [0], 55.5, "SURVEY.md §6 row 1 (55-56, 8 thr)"),
    ("data.cfg", 64, 3, 1, 0.0, 8, 20, main_coeffs, [0], 3.3, "SURVEY.md §6 row 2 (-Ofast)"),
    ("config2", 120, 3, 1, 0.0, 8, 5, main_coeffs, [0], 1.3, "SURVEY.md §6 row 4 (1.1-1.5)"),
    ("aniso.m sz128", 128, 1, 5, 0.8, 10, 20, demo_coeffs, [0, 1], 5.75, "SURVEY.md §6 row 6"),
    ("aniso.m sz256", 256, 1, 5, 0.8, 10, 20, demo_coeffs, [0, 1], 2.19, "SURVEY.md §6 row 7"),
]


def main():
    reps = 3
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    refalloc = "--refalloc" in sys.argv  # the reference's per-use heap vectors (oracle_set_reference_alloc)
    for name, sz, d, ks, g, ns, ml, coeffs, modes, ref_rate, src in CASES:
        o = Oracle(sz, d, ks, g, ns, 4, ml)
        o.set_reference_alloc(refalloc)
        xy = o.getNodes()
        ss, st = coeffs(xy)
        o.setCoeff(ss, st)
        u = gaussian(xy) * ss
        per = {}
        for m in modes:
            o.cache(m)
            o.mapping(u, m)  # warm-up
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                o.mapping(u, m)
                ts.append(time.perf_counter() - t0)
            per[m] = float(np.median(ts))
            o.uncache(m)
        o.close()
        rate = 1.0 / float(np.mean(list(per.values())))
        print(json.dumps({"case": name, "N": sz * sz * d * d, "modes": modes, "threads": threads,
                          "timing_mode": "reference_alloc" if refalloc else "port",
                          "oracle_apply_s": {str(k): round(v, 4) for k, v in per.items()},
                          "oracle_applies_per_s": round(rate, 3), "reference_applies_per_s": ref_rate,
                          "ratio_oracle_over_reference": round(rate / ref_rate, 2), "reference_source": src,
                          "cpu_model": cpu_model()}), flush=True)


if __name__ == "__main__":
    main()
