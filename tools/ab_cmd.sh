#!/bin/bash
# A/B of library builds ab/<name>.so (LIBS="prev new ...") on the driver's
# bench command itself (box 1080p8, two contexts), alternating processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  for L in ${LIBS:-prev new}; do
    PTAMD_LIB=ab/$L.so timeout -k 10 120 python3 bench.py --steps ${STEPS:-200} --warmup 10 --no-scene-legs --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abc_$L.$i.log 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/abc_$L.$i.log; exit 1; }
    echo "$L $(grep '^{' gpurun_out/abc_$L.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
  done
done
