#!/bin/bash
# round-5 GPU call 15: traversal grid share and refill threshold around the
# legs' settings (PT_OPT_WF_GRID = 20, PT_OPT_WF_REFILL = 21), frame-filling
# cameras and config 4 at (0,0,5); one process per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05r; mkdir -p $OUT
one() { # tag cam leg frames variant
  CAM=$2 LEG="$3" FRAMES=$4 REPS=2 timeout -k 10 300 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/grid.log
}
C4="sphere 3840 2160 16 8 1"; C3="sphere 1920 1080 8 4 3"; C5="synthetic:10000000 1920 1080 8 4 1"
for v in "g50r8@2:20=50,21=8" "g60r8@2:20=60,21=8" "g75r8@2:20=75,21=8" "g50r12@2:20=50,21=12" "g60r12@2:20=60,21=12" "g40r8@3:20=40,21=8"; do
  one c4ff scene "$C4" 4 "$v" || exit 1
done
for v in "g25r8@4:20=25,21=8" "g30r8@4:20=30,21=8" "g35r8@4:20=35,21=8" "g40r8@3:20=40,21=8" "g50r8@3:20=50,21=8" "g25r6@4:20=25,21=6"; do
  one c3ff scene "$C3" 12 "$v" || exit 1
done
for v in "g50r8@2:20=50,21=8" "g60r8@2:20=60,21=8" "g40r8@3:20=40,21=8"; do
  one c4ref reference "$C4" 6 "$v" || exit 1
done
for v in "g100@2:20=100" "g75r12@2:20=75,21=12" "g60r8@2:20=60,21=8"; do
  one c5ff scene "$C5" 6 "$v" || exit 1
done
