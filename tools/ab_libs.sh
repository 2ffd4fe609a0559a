#!/bin/bash
# A/B library builds ab/<name>.so (LIBS="prev new ..."), alternating processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  for L in ${LIBS:-prev new}; do
    PTAMD_LIB=ab/$L.so timeout -k 10 120 python3 tools/ab_bench.py --reps 10 ${AB_ARGS:-v:lds=1} > gpurun_out/ab_$L.$i.log 2>&1 || { echo "$L rc=$?"; cat gpurun_out/ab_$L.$i.log | tail -5; exit 1; }
    echo "$L $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$L.$i.log')); print({k: round(v['mean_ms'],4) for k,v in d['results'].items()})")"
  done
done
