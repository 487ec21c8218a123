set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "ANISO_EARLY_M2L=0" "ANISO_EARLY_M2L=1"; do
for wr in "8 0" "4 0" "2 0"; do
  env $cfg timeout -k 10 120 python tools/shard_time.py $wr > gpurun_out/shard.log 2>&1 || { tail -5 gpurun_out/shard.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/shard.log | cut -c1-200)"
done
done
