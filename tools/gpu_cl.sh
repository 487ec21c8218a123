set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "block or config3 or mapping_matches" --timeout 300 --timeout-method thread > gpurun_out/cl_tests.log 2>&1 || { tail -60 gpurun_out/cl_tests.log; exit 1; }
tail -1 gpurun_out/cl_tests.log
timeout -k 10 120 python tools/shard_time.py 8 0 > gpurun_out/shard.log 2>&1 || { tail -5 gpurun_out/shard.log; exit 1; }
tail -1 gpurun_out/shard.log
bash tools/ab_env.sh "ANISO_OVERLAP=0" "ANISO_OVERLAP=1" "ANISO_OVERLAP=0" "ANISO_OVERLAP=1"
