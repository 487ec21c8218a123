set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { tail -60 gpurun_out/gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/bench_check.log 2>&1 || { tail -20 gpurun_out/bench_check.log; exit 1; }
grep "^{" gpurun_out/bench_check.log | tail -1 | cut -c1-200
