#!/bin/bash
# r03u: phase 2 on the comm stream beside the early fine clusters; sharded / native tests, then timings
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "native or rehearsal or shard or clusters or fused or rccl" > gpurun_out/r03u/tests.log 2>&1 || { tail -40 gpurun_out/r03u/tests.log; exit 1; }
tail -2 gpurun_out/r03u/tests.log
for e in 1 0; do
  ANISO_EARLY_FINE=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 2 3 --native --no-timing > gpurun_out/r03u/n_e$e.log 2>&1 || { tail -20 gpurun_out/r03u/n_e$e.log; exit 1; }
  echo "early $e"; grep "^{" gpurun_out/r03u/n_e$e.log | cut -c1-100
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03u/tr -o run -- python3 tools/shard_time.py 8 0 --native --no-timing > gpurun_out/r03u/tr.log 2>&1 || { tail -20 gpurun_out/r03u/tr.log; exit 1; }
python3 tools/trace_last.py gpurun_out/r03u/tr/run_kernel_trace.csv
