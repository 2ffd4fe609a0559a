#!/bin/bash
# round-5 GPU call 21: frames per timed run of the scene legs (pipeline fill
# and drain amortised over more frames), the legs' settings otherwise
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05w; mkdir -p $OUT
one() { # tag cam leg frames variant
  CAM=$2 LEG="$3" FRAMES=$4 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 f$4 /" | tee -a $OUT/frames.log
}
C4="sphere 3840 2160 16 8 1"; C3="sphere 1920 1080 8 4 3"; C5="synthetic:10000000 1920 1080 8 4 1"
for f in 12 24 48; do
  one c3ref reference "$C3" $f "g25@4:20=25" || exit 1
  one c3ff scene "$C3" $f "g25@4:20=25" || exit 1
done
for f in 5 10 20; do
  one c5ref reference "$C5" $f "g33@3:20=33" || exit 1
done
for f in 6 12; do
  one c4ref reference "$C4" $f "g50@2:20=50" || exit 1
  one c4ff scene "$C4" $f "g50@2:20=50" || exit 1
done
