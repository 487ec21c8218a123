set -o pipefail
for c in 0 256 1024 2048; do
  ANISO_PTS_CAP=$c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cap_$c -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/cap_$c.log 2>&1 || exit 1
done
