#!/bin/bash
# round-5 GPU call 14: the tail kernel under frames in flight (PT_OPT_WF_TAIL
# = 17: -1 auto, 0 off), with its grid split like the traversal's (ab/tailgrid)
# or full (ab/cur); one process per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05p2; mkdir -p $OUT
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=2 PT_LEG_TAIL=1 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 $6 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/tail.log
}
for L in cur tailgrid; do
  one c4ff $L scene "sphere 3840 2160 16 8 1" 4 "t@2:20=50,17=-1" || exit 1
  one c4ref $L reference "sphere 3840 2160 16 8 1" 6 "t@2:20=50,17=-1" || exit 1
  one c3ref $L reference "sphere 1920 1080 8 4 3" 12 "t@4:20=25,17=-1" || exit 1
  one c5ref $L reference "synthetic:10000000 1920 1080 8 4 1" 6 "t@3:20=33,17=-1" || exit 1
done
one c4ff cur scene "sphere 3840 2160 16 8 1" 4 "off@2:20=50,17=0" || exit 1
one c4ref cur reference "sphere 3840 2160 16 8 1" 6 "off@2:20=50,17=0" || exit 1
