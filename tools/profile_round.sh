#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes.
# usage: bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
