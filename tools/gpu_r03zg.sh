#!/bin/bash
# r03zg: the per-mode stream's near field and corrections forked beside its M2L
# (main.cpp's mode-0 operator, config 4): whole -m gpu suite, then in-process A/B
# against ANISO_OVERLAP=0 (the previous serial schedule) at 1M and 4M points, one GPU
# and one rank of 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zg
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03zg/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03zg/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03zg/gpu_tests.log
timeout -k 10 300 python -u tools/ab_handles.py --ks 1 --reps 4 "" "ANISO_OVERLAP=0" > gpurun_out/r03zg/ab_ks1_w1.log 2>&1 || { tail -20 gpurun_out/r03zg/ab_ks1_w1.log; exit 1; }
grep "^{" gpurun_out/r03zg/ab_ks1_w1.log | cut -c1-330
timeout -k 10 400 python -u tools/ab_handles.py --ks 1 --sz 2048 --reps 3 "" "ANISO_OVERLAP=0" > gpurun_out/r03zg/ab_c4_w1.log 2>&1 || { tail -20 gpurun_out/r03zg/ab_c4_w1.log; exit 1; }
grep "^{" gpurun_out/r03zg/ab_c4_w1.log | cut -c1-330
timeout -k 10 400 python -u tools/ab_handles.py --ks 1 --sz 2048 --world 8 --reps 3 "" "ANISO_OVERLAP=0" > gpurun_out/r03zg/ab_c4_w8.log 2>&1 || { tail -20 gpurun_out/r03zg/ab_c4_w8.log; exit 1; }
grep "^{" gpurun_out/r03zg/ab_c4_w8.log | cut -c1-330
