#!/bin/bash
# A/B of two builds of the library on the 1M-point block matvec, in alternating
# processes (ANISO_LIB selects the build; "" = the in-tree library).
# usage: TAG=r05x REPS=3 bash tools/ab_libs.sh <libA|""> <libB|""> [ab_handles args...]
set -o pipefail
T=${TAG:-ab}
A=$1
B=$2
shift 2
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-3}); do
  for L in "$A" "$B"; do
    name=$([ -z "$L" ] && echo intree || basename "$(dirname "$L")")
    ANISO_LIB=$L timeout -k 10 200 python -u tools/ab_handles.py --reps 2 "$@" "" > gpurun_out/${T}_${name}_$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], d['best_ms'], d['stage_ms'])" gpurun_out/${T}_${name}_$r.log "$name.$r"
  done
done
