set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/ab_env.sh "ANISO_FUSE_SUB=1" "ANISO_FUSE_SUB=0" "ANISO_FUSE_SUB=1" "ANISO_FUSE_SUB=0"
