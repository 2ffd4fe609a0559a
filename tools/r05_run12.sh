#!/bin/bash
# round-5 GPU call 12: frame-filling cameras of configs 4/5 with two contexts
# (full grid, and half grid with the split-grid refill), one process each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05l; mkdir -p $OUT
one() {
  CAM=$2 LEG="$3" FRAMES=$4 REPS=2 timeout -k 10 300 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/ff.log
}
for v in g100@1: g100@2: g50@2:20=50; do one c5ff scene "synthetic:10000000 1920 1080 8 4 1" 6 $v || exit 1; done
for v in g100@1: g100@2: g50@2:20=50; do one c4ff scene "sphere 3840 2160 16 8 1" 4 $v || exit 1; done
for v in g25@4:20=25 g50@2:20=50 g100@2:; do one c4ref reference "sphere 3840 2160 16 8 1" 6 $v || exit 1; done
