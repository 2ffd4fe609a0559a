#!/bin/bash
# round-5 GPU call 20: occupancy and batching re-checked at the no-SLP build
# (fewer spills): box at 7 workgroups per CU (b7), wide flush loading 4
# candidates' records per trip (fb4), shading at 5 workgroups per CU (sh5),
# fb4+sh5; parity of all three together first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05v; mkdir -p $OUT
PTAMD_LIB=ab/all3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_all3.log 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_all3.log; exit 1; }
tail -1 $OUT/pytest_all3.log
LIBS="cur b7" REPS=3 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1 || { cat $OUT/ab_box.log; exit 1; }
cat $OUT/ab_box.log
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=2 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/legs.log
}
C3="sphere 1920 1080 8 4 3"
for i in 1 2; do
  for L in cur fb4 sh5 fb4sh5; do
    one c3ref $L reference "$C3" 12 "g25@4:20=25" || exit 1
    one c3ff $L scene "$C3" 12 "g25@4:20=25" || exit 1
  done
done
