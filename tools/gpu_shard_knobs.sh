# one rank-of-8 schedule (loopback, no stage events) under knob settings given as
# "NAME=VALUE ..." strings; each setting in its own process, twice, interleaved
set -o pipefail
T=${TAG:-r05}
for rep in 1 2; do
  for cfg in "$@"; do
    echo "## $cfg rep $rep"
    env $cfg timeout -k 10 300 python -u tools/shard_time.py 8 ${RANKS:-0 3} --native --no-timing || exit 1
  done
done > gpurun_out/${T}_knobs.log 2>&1
