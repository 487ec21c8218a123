set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/shard_times.log
for wr in "1 0" "2 0" "2 1" "4 0" "4 3" "8 0" "8 3" "8 7"; do
  timeout -k 10 120 python tools/shard_time.py $wr > gpurun_out/shard.log 2>&1 || { tail -5 gpurun_out/shard.log; exit 1; }
  tail -1 gpurun_out/shard.log | tee -a gpurun_out/shard_times.log
done
