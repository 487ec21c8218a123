#!/bin/bash
# r03s: full GPU suite; 8-shard rank times through the library's one-call matvec (loopback
# communicator) with and without the early fine clusters; kernel timeline of one
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
timeout -k 10 1000 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03s/tests.log 2>&1 || { tail -40 gpurun_out/r03s/tests.log; exit 1; }
tail -2 gpurun_out/r03s/tests.log
for e in 1 0; do
  ANISO_EARLY_FINE=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03s/native_e$e.log 2>&1 || { tail -20 gpurun_out/r03s/native_e$e.log; exit 1; }
  grep "^{" gpurun_out/r03s/native_e$e.log | cut -c1-160
done
timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --no-timing > gpurun_out/r03s/twophase.log 2>&1 || { tail -20 gpurun_out/r03s/twophase.log; exit 1; }
grep "^{" gpurun_out/r03s/twophase.log | cut -c1-160
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03s/tr -o run -- python3 tools/shard_time.py 8 0 --native --no-timing > gpurun_out/r03s/tr.log 2>&1 || { tail -20 gpurun_out/r03s/tr.log; exit 1; }
python3 tools/trace_last.py gpurun_out/r03s/tr/run_kernel_trace.csv
