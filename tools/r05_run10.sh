#!/bin/bash
# round-5 GPU call 10: wide-walk refill knobs under the legs' frames in flight
# (config 3 4 x 25 % at both cameras, config 5 3 x 33 % at (0,0,5)); one
# process per (library, leg), libraries ab/<name>.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05i; mkdir -p $OUT
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=1 timeout -k 10 240 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/knobs.log
}
for rep in 1 2; do
  for L in cur rf8 rf12 rf24 st8 st16; do
    one c3ref $L reference "sphere 1920 1080 8 4 3" 12 g25@4:20=25 || exit 1
    one c3ff $L scene "sphere 1920 1080 8 4 3" 8 g25@4:20=25 || exit 1
    one c5ref $L reference "synthetic:10000000 1920 1080 8 4 1" 6 g33@3:20=33 || exit 1
  done
done
