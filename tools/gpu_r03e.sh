#!/bin/bash
# r03e: fp64 16-RHS MFMA operator: parity tests, timing, counters, config-5 solve
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
  -k "fp64_mfma or fp32_mfma or config5 or batched or rebuilds_fp32" > gpurun_out/gpu_new_r03e.log 2>&1 || { tail -40 gpurun_out/gpu_new_r03e.log; exit 1; }
tail -14 gpurun_out/gpu_new_r03e.log
timeout -k 10 300 python -u tools/f64op_bench.py 1024 20 > gpurun_out/f64op_r03e.log 2>&1 || { tail -20 gpurun_out/f64op_r03e.log; exit 1; }
cat gpurun_out/f64op_r03e.log | grep "^{"
bash tools/f64op_prof.sh r03e || exit $?
timeout -k 10 300 python -u tools/config5.py > gpurun_out/config5_r03e.log 2>&1 || { tail -20 gpurun_out/config5_r03e.log; exit 1; }
tail -5 gpurun_out/config5_r03e.log
