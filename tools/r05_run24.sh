#!/bin/bash
# round-5 GPU call 24: config 3 at the frame-filling camera, grid share per
# context at the final build (4 x 25 / 30 / 35 %, 3 x 50 %), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05z; mkdir -p $OUT
one() { # tag cam leg frames variant
  CAM=$2 LEG="$3" FRAMES=$4 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/c3ff_grid.log
}
C3="sphere 1920 1080 8 4 3"
for i in 1 2; do
  for v in "g25@4:20=25" "g30@4:20=30" "g35@4:20=35" "g50@3:20=50"; do
    one c3ff scene "$C3" 12 "$v" || exit 1
  done
  for v in "g25@4:20=25" "g30@4:20=30"; do
    one c3ref reference "$C3" 12 "$v" || exit 1
  done
done
