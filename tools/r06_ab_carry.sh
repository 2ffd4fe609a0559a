#!/bin/bash
# A/B of drain compaction (PT_WIDE_CARRY) builds against the current build:
# frame-filling camera at the full grid, BASELINE's camera at config 3's leg
# grid (30 %), and the 10M cloud.  Frames are compared by digest.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export AB_TIMEOUT=${AB_TIMEOUT:-150}
L=${LIBS:-cur carry16 carry8 carry32}
LIBS="$L" AB_SCENES="sphere:6" AB_ITERS=2 tools/ab_libs_scenes.sh || exit 1
echo "-- refcam grid 30"
CAM=reference AB_ARGS="v:opt20=30" LIBS="$L" AB_SCENES="sphere:6" AB_ITERS=2 tools/ab_libs_scenes.sh || exit 1
LIBS="$L" AB_SCENES="random:10000000" AB_ITERS=1 tools/ab_libs_scenes.sh || exit 1
