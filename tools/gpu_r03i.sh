#!/bin/bash
# r03i: rehearsal with the config-4 leg, then the default bench (N=1) with every leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread -k "rehearsal" > gpurun_out/gpu_new_r03i.log 2>&1 || { tail -40 gpurun_out/gpu_new_r03i.log; exit 1; }
tail -4 gpurun_out/gpu_new_r03i.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03i.log 2>&1 || { tail -20 gpurun_out/bench_r03i.log; exit 1; }
grep "^{" gpurun_out/bench_r03i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('gmres',{}).get('steps_per_s'), d.get('block_solve'), d.get('config4'), d['cpu_baseline']['value'], d['speedup_vs_cpu'])"
