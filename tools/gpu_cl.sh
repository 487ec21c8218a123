set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
ANISO_LIB=aniso_amd/libaniso_probe.so timeout -k 10 300 python tools/tier_probe.py --block > gpurun_out/probe_block.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/probe_block.log | grep -E "tier|down|phase 3"
bash tools/ab_env.sh "ANISO_OVERLAP=1" "ANISO_OVERLAP=0" "ANISO_OVERLAP=1"
