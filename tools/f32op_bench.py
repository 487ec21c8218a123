"""Config 5's fp32 MFMA operator alone (16 right-hand sides, 1M points by default):
`steps` applies after a warm-up, for rocprofv3 kernel traces and PMC passes.
usage: f32op_bench.py [sz] [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import main_coeffs  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
a = aniso_amd.Aniso(sz, 1, 1, 0.8, 10, 4, 20)
a.setCoeff(*main_coeffs(a.getNodes()))
a.cache(0)
X = torch.rand(a.N, 16, device="cuda", dtype=torch.float32)
Y = torch.empty_like(X)
for _ in range(3):
    a.forward_f32_dev(X, Y)
torch.cuda.synchronize()
a.set_timing(True)
t0 = time.perf_counter()
for _ in range(steps):
    a.forward_f32_dev(X, Y)
torch.cuda.synchronize()
ms = 1e3 * (time.perf_counter() - t0) / steps
print(json.dumps({"N": a.N, "rhs": 16, "ms_per_apply": round(ms, 4),
                  "stage_ms": {k: round(v, 4) for k, v in a.stage_times().items()},
                  "fp32_cache_bytes": a.stats()["f32_cache_bytes"]}), flush=True)
