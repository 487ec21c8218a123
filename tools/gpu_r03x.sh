#!/bin/bash
# r03x: Krylov primitives (aniso_krylov_*), gmres_dist on them, block solve; bench legs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "krylov or gmres or solve or rehearsal" > gpurun_out/r03x/tests.log 2>&1 || { tail -40 gpurun_out/r03x/tests.log; exit 1; }
tail -2 gpurun_out/r03x/tests.log
timeout -k 10 300 python3 tools/probe_solve_iters.py > gpurun_out/r03x/probe.log 2>&1 || { tail -20 gpurun_out/r03x/probe.log; exit 1; }
cat gpurun_out/r03x/probe.log | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r03x/bench.log 2>&1 || { tail -20 gpurun_out/r03x/bench.log; exit 1; }
grep "^{" gpurun_out/r03x/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('block_solve'), d.get('gmres'))"
