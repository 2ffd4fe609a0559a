#!/bin/bash
# Native loop: GPU multi tests (2 and 3 streams), then the emulated root
# step at N = 8/4/2 on 2 against 3 render streams, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/native3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread -k native \
  > $OUT/multi.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/multi.log; exit 1; }
tail -1 $OUT/multi.log
for rep in 1 2; do
  for n in 8 4 2; do
    for st in 2 3; do
      PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-scene-legs --steps 400 --streams $st \
        > $OUT/n${n}_st${st}_$rep.log 2>&1 || { echo "rc=$? n=$n st=$st"; tail -5 $OUT/n${n}_st${st}_$rep.log; exit 1; }
      echo "n=$n streams=$st rep=$rep $(grep '^{' $OUT/n${n}_st${st}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["step_loop"])')"
    done
  done
done
