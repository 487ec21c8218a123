#!/bin/bash
# Whole-round GPU check: parity tests, smoke(), default bench (with the CPU leg),
# bench kernel trace + stats + PMC traffic, config 5's MFMA operator counters and the
# per-rank shard times.  Every GPU step has its own limit; the first failure ends it.
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
grep "^{" gpurun_out/bench_$TAG.log | cut -c1-300
bash tools/gpu_prof.sh $TAG || exit $?
bash tools/f32op_prof.sh $TAG || exit $?
for w in 1 8; do
  timeout -k 10 200 python -u tools/shard_time.py $w 0 >> gpurun_out/shard_$TAG.log 2>&1 || { tail -20 gpurun_out/shard_$TAG.log; exit 1; }
done
grep "^{" gpurun_out/shard_$TAG.log
