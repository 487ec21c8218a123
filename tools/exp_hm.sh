#!/bin/bash
# Harmonic-kernel experiments: parity tests, then A/B over ANISO_HM_VAR (bit 0 XCD
# order, bit 1 one Newton step, bit 2 four waves per SIMD).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || { tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -2 gpurun_out/exp_tests.log
ANISO_HM_VAR=3 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "harmonic or block or config3" --timeout 300 --timeout-method thread > gpurun_out/exp_tests_v3.log 2>&1 || { tail -30 gpurun_out/exp_tests_v3.log; exit 1; }
tail -2 gpurun_out/exp_tests_v3.log
bash tools/ab_env.sh "ANISO_HM_VAR=0" "ANISO_HM_VAR=1" "ANISO_HM_VAR=2" "ANISO_HM_VAR=3" "ANISO_HM_VAR=4" "ANISO_HM_VAR=7" "ANISO_HM_VAR=0"
