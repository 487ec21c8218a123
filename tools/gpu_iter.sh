#!/bin/bash
# one GPU iteration: parity tests, bench, kernel trace (usage: bash tools/gpu_iter.sh <tag>)
set -o pipefail
TAG=${1:-it}
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_$TAG.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || exit $?
