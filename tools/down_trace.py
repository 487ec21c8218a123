"""Per-task phase timeline of the down pass (k_down_tier) on a -DANISO_DOWN_TRACE build
(tools/build_variant.sh downtrace "-DANISO_DOWN_TRACE=1", then ANISO_LIB=build/ab_downtrace/
libaniso_mi355x.so): the 100 MHz wall clock at each task's start and after its four
phases [task records + locals loads, L2L chain from level 1, task levels, owned
points].  Prints the launch span and the phases' medians in microseconds.
usage: down_trace.py [SZ]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import aniso_amd  # noqa: E402
from bench import demo_coeffs  # noqa: E402

sz = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
op = aniso_amd.Aniso(sz, 1, 5, 0.8, 10, 4, 20)
xy = op.getNodes()
op.setCoeff(*demo_coeffs(xy))
for m in range(9):
    op.cache(m)
x = torch.rand(5, op.N, dtype=torch.float64, device="cuda")
y = torch.zeros_like(x)
for _ in range(4):
    op.block_op_dev(2, x, y, tree=True)
torch.cuda.synchronize()
ntask = op.stats()["leaves"] // 16
lib = aniso_amd.lib()
fn = lib.aniso_debug_down_trace
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(min(ntask, 16384) * 6, dtype=np.int64)
assert fn(buf.ctypes.data, min(ntask, 16384)) == 0
t = buf.reshape(-1, 6)[:, :5].astype(np.float64) / 100.0  # 100 MHz ticks -> us
t0 = t[:, 0].min()
ph = np.diff(t, axis=1)
print(json.dumps({"tasks": int(t.shape[0]), "launch_us": round(float(t[:, 4].max() - t0), 2),
                  "phase_us_p50": [round(float(v), 2) for v in np.median(ph, axis=0)],
                  "task_us_p50": round(float(np.median(t[:, 4] - t[:, 0])), 2),
                  "start_us_p90": round(float(np.percentile(t[:, 0] - t0, 90)), 2)}))
