#!/bin/bash
# r03aa: down-pass phase 0 in two independent rounds: parity of the apply/block/shard tests, timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03aa
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "block or shard or stages or mapping or config3 or oracle or forward" > gpurun_out/r03aa/tests.log 2>&1 || { tail -40 gpurun_out/r03aa/tests.log; exit 1; }
tail -2 gpurun_out/r03aa/tests.log
for r in 1 2; do timeout -k 10 200 python -u tools/ab_timing.py 60 2>&1 | grep "^{"; done
timeout -k 10 200 python3 tools/shard_time.py 8 0 1 --native --no-timing 2>&1 | grep "^{" | cut -c1-90
