set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
ANISO_TOP_SPAN=2 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "config3 or block or shard" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_span.log 2>&1 || { tail -60 gpurun_out/gpu_tests_span.log; exit 1; }
tail -1 gpurun_out/gpu_tests_span.log
bash tools/ab_env.sh "ANISO_OVERLAP=1" "ANISO_TOP_SPAN=2" "ANISO_TOP_SPAN=1" "ANISO_TOP_SPAN=3" "ANISO_OVERLAP=0"
