set -o pipefail
for v in "ANISO_SYMMETRIC=0" "ANISO_MAX_CANON=0" "ANISO_MAX_CANON=4" "ANISO_MAX_CANON=8" "ANISO_MAX_CANON=16" "ANISO_MAX_CANON=32"; do
  env $v timeout -k 10 120 python bench.py --no-cpu --steps 20 > gpurun_out/exp_$v.log 2>&1 || exit 1
done
