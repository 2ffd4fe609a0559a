#!/bin/bash
# round-5 GPU call 3: frames in flight x traversal grid for the scene legs,
# one variant per process (a process's least-priority streams share
# GPU_MAX_HW_QUEUES hardware queues, so variants must not coexist)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05c; mkdir -p $OUT
one() { # tag cam leg frames variant
  CAM=$2 LEG="$3" FRAMES=$4 REPS=2 timeout -k 10 240 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/legs.log
}
for rep in 1 2; do
  for v in g100@3: g100@2: g100@4: g50@2:20=50 g33@3:20=33 g25@4:20=25; do one c3ref reference "sphere 1920 1080 8 4 3" 12 $v || exit 1; done
  for v in g100@3: g50@2:20=50 g25@4:20=25; do one c3scene scene "sphere 1920 1080 8 4 3" 12 $v || exit 1; done
  for v in g100@1: g100@2: g50@2:20=50 g33@3:20=33; do one c5ref reference "synthetic:10000000 1920 1080 8 4 1" 6 $v || exit 1; done
  for v in g100@1: g50@2:20=50; do one c5scene scene "synthetic:10000000 1920 1080 8 4 1" 4 $v || exit 1; done
done
