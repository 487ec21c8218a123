#!/bin/bash
# r03a: the new GPU tests first, then the whole suite, then a quick bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 \
  -k "time_out or rebuilds_fp32 or repeat_its_begin or staged or clusters_match or knobs or fused_top or config3_size or full_size_odd or sz512" > gpurun_out/gpu_new_r03a.log 2>&1 || { tail -40 gpurun_out/gpu_new_r03a.log; exit 1; }
tail -20 gpurun_out/gpu_new_r03a.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 > gpurun_out/gpu_tests_r03a.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03a.log; exit 1; }
tail -14 gpurun_out/gpu_tests_r03a.log
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench_r03a.log 2>&1 || { tail -20 gpurun_out/bench_r03a.log; exit 1; }
grep "^{" gpurun_out/bench_r03a.log | cut -c1-400
