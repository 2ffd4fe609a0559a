#!/bin/bash
# Emulated root step (PT_BENCH_EMULATE_RANKS) on the native loop: render
# streams from torch's pool (PT_BENCH_NATIVE_TORCH_STREAMS=1) against the
# library's own least-priority streams (=0), alternating, 2 runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/native_streams
mkdir -p $OUT
for n in ${NS:-8 4 2}; do
  for rep in 1 2; do
    for ts in 1 0; do
      PT_BENCH_EMULATE_RANKS=$n PT_BENCH_NATIVE_TORCH_STREAMS=$ts timeout -k 10 200 \
        python -u bench.py --no-cpu-baseline --no-scene-legs --steps ${STEPS:-400} ${EXTRA:-} > $OUT/n${n}_ts${ts}_$rep.log 2>&1 \
        || { echo "rc=$? n=$n ts=$ts"; tail -5 $OUT/n${n}_ts${ts}_$rep.log; exit 1; }
      echo "n=$n torch_streams=$ts rep=$rep $(grep '^{' $OUT/n${n}_ts${ts}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("step_loop"))')"
    done
  done
done
