set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "config4_four" --timeout 300 --timeout-method thread --durations=3 > gpurun_out/c4_tests.log 2>&1 || { tail -60 gpurun_out/c4_tests.log; exit 1; }
grep -E "passed|failed|s call" gpurun_out/c4_tests.log | tail -4
