set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=8 > gpurun_out/gpu_tests_final.log 2>&1 || { tail -60 gpurun_out/gpu_tests_final.log; exit 1; }
tail -12 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
bash tools/gpu_prof.sh r01j || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r01j.log 2>&1 || { tail -20 gpurun_out/bench_r01j.log; exit 1; }
grep "^{" gpurun_out/bench_r01j.log | tail -1 | cut -c1-400
