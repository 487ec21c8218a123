set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "harmonic or block or config3" --timeout 300 --timeout-method thread > gpurun_out/cl_tests.log 2>&1 || { tail -40 gpurun_out/cl_tests.log; exit 1; }
tail -3 gpurun_out/cl_tests.log
bash tools/ab_env.sh "ANISO_HM_CLUSTER=1" "ANISO_HM_CLUSTER=0" "ANISO_HM_VAR=6"
