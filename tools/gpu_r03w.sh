#!/bin/bash
# r03w: register-held CGS2 sweeps + the next matvec ahead of the host's Givens step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "solve or gmres" > gpurun_out/r03w/tests.log 2>&1 || { tail -40 gpurun_out/r03w/tests.log; exit 1; }
tail -2 gpurun_out/r03w/tests.log
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r03w/bench.log 2>&1 || { tail -20 gpurun_out/r03w/bench.log; exit 1; }
grep "^{" gpurun_out/r03w/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('block_solve'), d.get('gmres'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03w/tr -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r03w/tr.log 2>&1 || { tail -20 gpurun_out/r03w/tr.log; exit 1; }
grep -E "k_cgs|k_mdot|k_maxpy|k_scale_rsqrt" gpurun_out/r03w/tr/run_kernel_stats.csv | cut -c1-160
