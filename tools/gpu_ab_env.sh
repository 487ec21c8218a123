#!/bin/bash
# A/B of environment settings on the 1-GPU bench and one 8-way shard:
# usage: gpu_ab_env.sh "VAR=a" "VAR=b" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for kv in "$@"; do
  for rep in 1 2; do
    env $kv timeout -k 10 200 python3 bench.py --no-cpu --steps 30 --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$kv bench: $(grep '^{' gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"])')"
  done
  env $kv timeout -k 10 200 python3 tools/shard_time.py 8 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "$kv shard8: $(grep '^{' gpurun_out/ab.log | cut -c1-230)"
done
