#!/bin/bash
# Kernel trace of one rank of an 8-way sharded block matvec (tools/shard_time.py).
set -o pipefail
TAG=${1:-sp}
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0; do
  ANISO_EARLY_M2L=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shardprof_${TAG}_$v -o run -- python3 tools/shard_time.py 8 0 > gpurun_out/shardprof_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/shardprof_${TAG}_$v.log; exit 1; }
  grep "^{" gpurun_out/shardprof_${TAG}_$v.log
done
