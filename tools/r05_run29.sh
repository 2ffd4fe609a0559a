#!/bin/bash
# round-5 GPU call 29: pixels per thread of the culled fill / assembly
# workgroups (PT_PIX_PER_FILL 8 / 16 / 32: fewer trailing workgroups), box on
# the driver's command (200 frames) and the config-5 leg at (0,0,5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zf; mkdir -p $OUT
LIBS="fill fill16 fill32" REPS=3 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1 || { cat $OUT/ab_box.log; exit 1; }
cat $OUT/ab_box.log
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/legs.log
}
for L in fill fill16 fill32 fill fill16 fill32; do
  one c5ref $L reference "synthetic:10000000 1920 1080 8 4 1" 12 "g33@3:20=33" || exit 1
done
