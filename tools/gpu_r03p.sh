#!/bin/bash
# r03p: kernel timeline of one 8-shard block matvec (rank 0) without stage events; times with and without them
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --no-timing > gpurun_out/r03p/nt.log 2>&1 || { tail -20 gpurun_out/r03p/nt.log; exit 1; }
timeout -k 10 200 python3 tools/shard_time.py 8 0 1 > gpurun_out/r03p/t.log 2>&1 || { tail -20 gpurun_out/r03p/t.log; exit 1; }
grep "^{" gpurun_out/r03p/nt.log gpurun_out/r03p/t.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03p/w8nt -o run -- python3 tools/shard_time.py 8 0 --no-timing > gpurun_out/r03p/w8nt.log 2>&1 || { tail -20 gpurun_out/r03p/w8nt.log; exit 1; }
python3 tools/trace_last.py gpurun_out/r03p/w8nt/run_kernel_trace.csv
