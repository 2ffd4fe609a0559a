#!/bin/bash
# round-5 GPU call 16: the device code built without LLVM's SLP vectorizer
# (ab/noslp.so, -fno-slp-vectorize: no v_pk_*_f32, fewer moves and spills)
# against the same source built as now (ab/base.so): parity first, then the
# box on the driver's command (200 frames) and the legs, alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05s; mkdir -p $OUT
PTAMD_LIB=ab/noslp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_noslp.log 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_noslp.log; exit 1; }
tail -2 $OUT/pytest_noslp.log
LIBS="base noslp" REPS=3 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1 || { cat $OUT/ab_box.log; exit 1; }
cat $OUT/ab_box.log
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=2 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/legs.log
}
C4="sphere 3840 2160 16 8 1"; C3="sphere 1920 1080 8 4 3"; C5="synthetic:10000000 1920 1080 8 4 1"
for i in 1 2; do
  for L in base noslp; do
    one c3ref $L reference "$C3" 12 "g25@4:20=25" || exit 1
    one c3ff $L scene "$C3" 12 "g25@4:20=25" || exit 1
    one c5ref $L reference "$C5" 6 "g33@3:20=33" || exit 1
  done
done
for L in base noslp; do
  one c4ref $L reference "$C4" 6 "g50@2:20=50" || exit 1
done
