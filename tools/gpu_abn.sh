#!/bin/bash
# same-box A/B of several library builds (cur = in-tree, others = build/ab_<name>):
# serial stage times and the overlapped block matvec.  usage: tools/gpu_abn.sh name1 name2 ...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
for L in cur "$@"; do
  if [ $L = cur ]; then LIB=$PWD/aniso_amd/libaniso_mi355x.so; else LIB=$PWD/build/ab_$L/libaniso_mi355x.so; fi
  ANISO_LIB=$LIB ANISO_OVERLAP=0 timeout -k 10 200 python -u bench.py --no-cpu --steps 30 2>&1 | grep "^{" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L serial', d['value'], {k: d['stage_ms'][k] for k in ('up', 'm2l', 'near', 'down')})" || exit 1
  ANISO_LIB=$LIB timeout -k 10 200 python -u tools/ab_timing.py 60 | sed "s/^/$L overlapped /" || exit 1
done
done
