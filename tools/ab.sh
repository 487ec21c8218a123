#!/bin/bash
# A/B on one box: bash tools/ab.sh "ENV_A" "ENV_B" [reps]; alternates the two bench runs
set -o pipefail
A=$1; B=$2; R=${3:-2}
for i in $(seq 1 $R); do
  for v in "$A" "$B"; do
    env $v timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 5 > gpurun_out/ab.log 2>&1 || exit 1
    python -c "import json; d=[json.loads(l) for l in open('gpurun_out/ab.log') if l.startswith('{')][0]; print('$v', d['value'], {k: round(x,4) for k,x in d['stage_ms'].items()})" >> gpurun_out/ab_summary.txt
  done
done
