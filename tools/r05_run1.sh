#!/bin/bash
# round-5 GPU call 1: checks, gather ceilings, driver bench, box A/B, grid A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r05_check.sh || exit $?
LIBS="prev new new2" REPS=3 bash tools/ab_cmd.sh > gpurun_out/r05a/ab_box.log 2>&1; cat gpurun_out/r05a/ab_box.log
for cam in reference scene; do
  CAM=$cam LEG="sphere 1920 1080 8 4 3" FRAMES=12 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py g100: g50:20=50 g33:20=33 > gpurun_out/r05a/grid_ab_$cam.log 2>&1 || { echo "grid ab rc=$?"; tail -5 gpurun_out/r05a/grid_ab_$cam.log; exit 1; }
  cat gpurun_out/r05a/grid_ab_$cam.log
done
