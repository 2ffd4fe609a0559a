#!/bin/bash
# round-5 GPU call 37: the wavefront pipeline's pixel mapping from the item
# origins, a 32-bit path quotient in wf_gen and fold_one in wf_fold: parity,
# config and wavefront GPU tests on the product build, then the legs at
# (0,0,5) and config 3 frame-filling against the previous build (ab/cur.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zn; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_group.py tests/test_gpu_multi.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/legs.log
}
for L in cur wfo cur wfo; do
  one c3ref $L reference "sphere 1920 1080 8 4 3" 12 "g30@4:20=30" || exit 1
  one c5ref $L reference "synthetic:10000000 1920 1080 8 4 1" 12 "g33@3:20=33" || exit 1
  one c3ff $L scene "sphere 1920 1080 8 4 3" 12 "g30@4:20=30" || exit 1
done
