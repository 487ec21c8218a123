#!/bin/bash
# r03zk: the near field back at 132 VGPRs / 3 waves per SIMD by default (ANISO_NEAR_WPE=3;
# with the dynamic target hand-out the 128-VGPR cap measured 2.6 % slower, r03zj):
# in-process A/B, whole -m gpu suite, kernel trace + stats, FETCH/WRITE passes, bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zk
timeout -k 10 400 python -u tools/ab_handles.py --reps 4 "" "ANISO_NEAR_WPE=4" > gpurun_out/r03zk/ab_w1.log 2>&1 || { tail -20 gpurun_out/r03zk/ab_w1.log; exit 1; }
grep "^{" gpurun_out/r03zk/ab_w1.log | cut -c1-300
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03zk/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03zk/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03zk/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zk/smoke.log 2>&1 || { tail -20 gpurun_out/r03zk/smoke.log; exit 1; }
bash tools/profile_round.sh r03zk > /dev/null || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03zk/fetch/run_counter_collection.csv gpurun_out/prof_r03zk/write/run_counter_collection.csv gpurun_out/r03zk/pmc_summary.json > /dev/null || exit 1
python3 tools/trace_last.py gpurun_out/prof_r03zk/trace/run_kernel_trace.csv > gpurun_out/r03zk/timeline_w1.txt || exit 1
cat gpurun_out/r03zk/timeline_w1.txt
timeout -k 10 600 python bench.py > gpurun_out/r03zk/bench.log 2>&1 || { tail -20 gpurun_out/r03zk/bench.log; exit 1; }
grep "^{" gpurun_out/r03zk/bench.log | tail -1 | cut -c1-300
