#!/bin/bash
# round-5 GPU call 11: the runtime refill threshold (PT_OPT_WF_REFILL = 21)
# per leg setting; one process per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05j; mkdir -p $OUT
one() {
  CAM=$2 LEG="$3" FRAMES=$4 REPS=1 timeout -k 10 240 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/refill.log
}
for rep in 1 2; do
  for r in 4 6 8 12 16; do :; done
  for r in 4 6 8 12 16; do
    one c3ref reference "sphere 1920 1080 8 4 3" 12 "r${r}@4:20=25,21=$r" || exit 1
    one c3ff scene "sphere 1920 1080 8 4 3" 8 "r${r}@4:20=25,21=$r" || exit 1
  done
  [ $rep = 2 ] && break
  for r in 4 8 16; do
    one c5ref reference "synthetic:10000000 1920 1080 8 4 1" 6 "r${r}@3:20=33,21=$r" || exit 1
    one c4ref reference "sphere 3840 2160 16 8 1" 2 "r${r}@3:20=33,21=$r" || exit 1
  done
  for r in 8 12 16; do
    one c5ff scene "synthetic:10000000 1920 1080 8 4 1" 3 "r${r}@1:21=$r" || exit 1
    one c4ff scene "sphere 3840 2160 16 8 1" 2 "r${r}@1:21=$r" || exit 1
  done
done
