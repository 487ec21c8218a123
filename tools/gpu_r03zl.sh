#!/bin/bash
# r03zl: every rank of 8 at the round's close (loopback communicator: one rank's
# one-call schedule on one GPU, tools/shard_time.py --native), 1M block matvec
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03zl
timeout -k 10 500 python3 -u tools/shard_time.py 8 0 1 2 3 4 5 6 7 --native --no-timing > gpurun_out/r03zl/w8.log 2>&1 || { tail -20 gpurun_out/r03zl/w8.log; exit 1; }
grep '^{' gpurun_out/r03zl/w8.log | cut -c1-120
