#!/bin/bash
# A/B of environment knobs on the bench (no CPU baseline). usage: bash tools/ab_env.sh "ENV=1" "ENV=2" ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu --steps 10 > "gpurun_out/ab_${cfg// /_}.log" 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['stage_ms'])" "gpurun_out/ab_${cfg// /_}.log" "$cfg"
done
