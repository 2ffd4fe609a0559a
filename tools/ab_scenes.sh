#!/bin/bash
# A/B of library builds ab/<name>.so (LIBS) on several scenes (SCENES, ab_bench
# --scene values), alternating processes, ROUNDS rounds.  Prints mean ms per frame.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sc in ${SCENES:-sphere:6}; do
  for i in $(seq 1 ${ROUNDS:-2}); do
    for L in ${LIBS:-base new}; do
      PTAMD_LIB=ab/$L.so timeout -k 10 200 python3 tools/ab_bench.py --scene $sc --reps ${REPS:-3} ${AB_EXTRA:-} v:lds=0 > gpurun_out/ab_${L}_$i.log 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/ab_${L}_$i.log; exit 1; }
      echo "$sc $L $(python3 -c "import json; d=json.load(open('gpurun_out/ab_${L}_$i.log')); print({k: round(v['mean_ms'],3) for k,v in d['results'].items()})")"
    done
  done
done
