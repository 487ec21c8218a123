#!/bin/bash
# r03d: block solve + sharded-GMRES bench legs + the changed tests, then the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
  -k "block_solve or clusters_match or small_clusters or knobs or sharded_apply_composes or tree_order_paths or rehearsal" > gpurun_out/gpu_new_r03d.log 2>&1 || { tail -40 gpurun_out/gpu_new_r03d.log; exit 1; }
tail -14 gpurun_out/gpu_new_r03d.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03d.log 2>&1 || { tail -20 gpurun_out/bench_r03d.log; exit 1; }
grep "^{" gpurun_out/bench_r03d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('gmres'), d.get('block_solve'), d['cpu_baseline'], d['rel_err_vs_cpu_detail'], d['speedup_vs_cpu'])"
