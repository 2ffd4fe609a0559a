#!/bin/bash
# round-5 GPU call 4: config 4 frames in flight (one variant per process);
# emulated 1/8 shares of configs 4/5 at the reference camera, grid 100 vs 1/C
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05d; mkdir -p $OUT
one() {
  CAM=$2 LEG="$3" FRAMES=$4 REPS=2 timeout -k 10 240 python3 tools/r05_leg_ab.py "$5" > $OUT/tmp.log 2>&1 || { echo "$1 $5 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 /" | tee -a $OUT/legs.log
}
for v in g100@1: g50@2:20=50 g100@2:; do one c4ref reference "sphere 3840 2160 16 8 1" 3 $v || exit 1; done
for cfg in config4 config5; do
  for g in 100 33; do
    CAM=reference GRID=$g timeout -k 10 300 python3 tools/r04_scene_emu.py $cfg 8 3 > $OUT/emu_${cfg}_g$g.log 2>&1 || { echo "emu $cfg $g rc=$?"; tail -5 $OUT/emu_${cfg}_g$g.log; exit 1; }
    grep '^{' $OUT/emu_${cfg}_g$g.log | cut -c1-600
  done
done
