#!/bin/bash
# round-5 GPU call 2: box fold/skip variants on the driver's command; grid x contexts on configs 3/4/5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05b; mkdir -p $OUT
LIBS="prev e2 e32 e12 e123" REPS=3 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1; cat $OUT/ab_box.log
run() { # name cam leg frames variants...
  local tag=$1 cam=$2 leg=$3 fr=$4; shift 4
  CAM=$cam LEG="$leg" FRAMES=$fr REPS=2 timeout -k 10 420 python3 tools/r05_leg_ab.py "$@" > $OUT/grid_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 $OUT/grid_$tag.log; exit 1; }
  cat $OUT/grid_$tag.log
}
run c3ref reference "sphere 1920 1080 8 4 3" 12 g100@3: g33@3:20=33 g25@3:20=25 g20@3:20=20 g50@2:20=50 g25@4:20=25
run c5ref reference "synthetic:10000000 1920 1080 8 4 1" 6 g100@1: g50@2:20=50 g33@3:20=33
# config 4: one variant per process (55 GB of path buffers per context)
for v in g100@1: g50@2:20=50 g33@3:20=33; do run c4ref_${v%%:*} reference "sphere 3840 2160 16 8 1" 3 $v; done
