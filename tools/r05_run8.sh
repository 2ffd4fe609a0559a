#!/bin/bash
# round-5 GPU call 8: wide-kernel lane counters at grid 100/25; frames in
# flight x grid sweep at the frame-filling cameras and wider at (0,0,5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05g; mkdir -p $OUT
bash tools/r05_wide_counters.sh
one() {
  CAM=$2 LEG="$3" FRAMES=$4 REPS=2 timeout -k 10 240 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/legs.log
}
for v in g25@4:20=25 g16@6:20=16 g20@5:20=20; do one c3ref reference "sphere 1920 1080 8 4 3" 12 $v || exit 1; done
for v in g33@3:20=33 g25@4:20=25 g16@6:20=16; do one c3scene scene "sphere 1920 1080 8 4 3" 8 $v || exit 1; done
for v in g100@1: g33@3:20=33 g25@4:20=25; do one c5scene scene "synthetic:10000000 1920 1080 8 4 1" 4 $v || exit 1; done
for v in g100@1: g33@3:20=33; do one c4scene scene "sphere 3840 2160 16 8 1" 2 $v || exit 1; done
timeout -k 10 200 python3 tools/r05_box_order.py 20 15 o00 o11 o01 o10 > $OUT/box_order20.log 2>&1 && cat $OUT/box_order20.log
timeout -k 10 200 python3 tools/r05_box_order.py 200 5 o00 o11 > $OUT/box_order200.log 2>&1 && cat $OUT/box_order200.log
