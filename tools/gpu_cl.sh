set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "harmonic or block or config3" --timeout 300 --timeout-method thread > gpurun_out/cl_tests.log 2>&1 || { tail -40 gpurun_out/cl_tests.log; exit 1; }
tail -3 gpurun_out/cl_tests.log
ANISO_HM_VAR=12 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "clusters" --timeout 300 --timeout-method thread > gpurun_out/cl_tests_pf.log 2>&1 || { tail -40 gpurun_out/cl_tests_pf.log; exit 1; }
tail -1 gpurun_out/cl_tests_pf.log
bash tools/ab_env.sh "ANISO_HM_VAR=4" "ANISO_HM_VAR=12" "ANISO_HM_VAR=28" "ANISO_HM_VAR=20" "ANISO_HM_VAR=36"
