#!/bin/bash
# round 6: A/B of two library builds (ab/$A.so, ab/$B.so) on scene legs as
# bench.py times them (--leg: contexts and grid of SCENE_LEGS), alternating
# processes: LEGS="config3:ref config5:ref" A=smax0 B=smax1 tools/r06_ab_legs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06o}; mkdir -p $OUT
for leg in ${LEGS:-config3:ref config3:ff config4:ref config5:ref}; do
  key=${leg%%:*}; cam=${leg#*:}
  for rep in $(seq 1 ${REPS:-3}); do
    for L in ${A:-smax0} ${B:-smax1}; do
      PTAMD_LIB=ab/$L.so timeout -k 10 300 python bench.py --leg $key --leg-camera $cam --steps ${STEPS:-24} > $OUT/${key}_${cam}_${L}_$rep.log 2>&1 || { echo "$L rc=$?"; tail -5 $OUT/${key}_${cam}_${L}_$rep.log; exit 1; }
      echo "$key $cam $L $(tail -1 $OUT/${key}_${cam}_${L}_$rep.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
