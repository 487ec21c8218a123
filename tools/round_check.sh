#!/bin/bash
# Full GPU check for one round: parity tests, default bench (with CPU baseline),
# kernel trace + stats, PMC passes. usage: bash tools/round_check.sh <tag>
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
bash tools/profile_round.sh $TAG
