#!/bin/bash
# r03g: the library's own exchange (native comm) tests, one-rank RCCL A/B, per-rank times
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
  -k "native_exchange or rehearsal or rccl" > gpurun_out/gpu_new_r03g.log 2>&1 || { tail -40 gpurun_out/gpu_new_r03g.log; exit 1; }
tail -8 gpurun_out/gpu_new_r03g.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29541 tools/comm_ab.py > gpurun_out/comm_ab_r03g.log 2>&1 || { tail -20 gpurun_out/comm_ab_r03g.log; exit 1; }
grep "^{" gpurun_out/comm_ab_r03g.log
bash tools/gpu_r03f.sh
