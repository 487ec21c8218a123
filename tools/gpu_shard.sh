#!/bin/bash
# Sharded-apply check: the two-phase parity tests, per-rank shard times at 1/2/4/8
# ranks, and the bench. usage: bash tools/gpu_shard.sh <tag> "<pytest -k expr>"
set -o pipefail
TAG=${1:-s}
EXPR=${2:-"two_phase or eight_shards or rehearsal"}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$EXPR" --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
for w in 1 2 4 8; do
  timeout -k 10 200 python -u tools/shard_time.py $w 0 >> gpurun_out/shard_$TAG.log 2>&1 || { tail -20 gpurun_out/shard_$TAG.log; exit 1; }
done
cat gpurun_out/shard_$TAG.log | grep "^{"
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
grep "^{" gpurun_out/bench_$TAG.log | cut -c1-600
