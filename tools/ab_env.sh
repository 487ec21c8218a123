export TMPDIR=/tmp
for cfg in "X=1" "ANISO_SYMMETRIC=0" "ANISO_MAX_CANON=16" "X=2"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu --steps 10 > gpurun_out/ab_$cfg.log 2>&1 || exit $?
done
