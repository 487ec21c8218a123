#!/bin/bash
# Quick GPU iteration: selected parity tests (pytest -k EXPR) then the bench
# without the CPU baseline. usage: bash tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args]
set -o pipefail
TAG=${1:-q}
EXPR=${2:-block}
shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$EXPR" --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu "$@" > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.log
