set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 2 3 4; do ANISO_NEAR_VAR=$v timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "harmonic_block_apply or config3_size_matches" --timeout 200 --timeout-method thread > gpurun_out/nv_tests_$v.log 2>&1 || { tail -30 gpurun_out/nv_tests_$v.log; exit 1; }; tail -1 gpurun_out/nv_tests_$v.log; done
bash tools/ab_env.sh "ANISO_NEAR_VAR=0 ANISO_OVERLAP=0" "ANISO_NEAR_VAR=1 ANISO_OVERLAP=0" "ANISO_NEAR_VAR=2 ANISO_OVERLAP=0" "ANISO_NEAR_VAR=3 ANISO_OVERLAP=0" "ANISO_NEAR_VAR=4 ANISO_OVERLAP=0" "ANISO_NEAR_VAR=0" "ANISO_NEAR_VAR=3" "ANISO_NEAR_VAR=4"
