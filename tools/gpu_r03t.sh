#!/bin/bash
# r03t: upper-cluster size, with and without the early fine clusters (8 shards, loopback one-call matvec)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
for ud in 2 1 0; do
 for e in 1 0; do
  ANISO_HM_UPPER_DEPTH=$ud ANISO_EARLY_FINE=$e timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing > gpurun_out/r03t/n_ud${ud}_e$e.log 2>&1 || { tail -20 gpurun_out/r03t/n_ud${ud}_e$e.log; exit 1; }
  echo "upper_depth $ud early $e"; grep "^{" gpurun_out/r03t/n_ud${ud}_e$e.log | cut -c1-100
 done
done
for ud in 2 1; do
  ANISO_HM_UPPER_DEPTH=$ud timeout -k 10 200 python3 tools/shard_time.py 1 0 > gpurun_out/r03t/w1_ud$ud.log 2>&1 || { tail -20 gpurun_out/r03t/w1_ud$ud.log; exit 1; }
  echo "world 1 upper_depth $ud"; grep "^{" gpurun_out/r03t/w1_ud$ud.log | cut -c1-100
done
ANISO_TOP_TRACE=1 ANISO_HM_UPPER_DEPTH=1 timeout -k 10 200 python3 -u tools/top_trace.py 8 0 --native > gpurun_out/r03t/trace_e1.log 2>&1 || { tail -20 gpurun_out/r03t/trace_e1.log; exit 1; }
grep "^{" gpurun_out/r03t/trace_e1.log | cut -c1-900
