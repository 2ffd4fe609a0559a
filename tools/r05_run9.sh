#!/bin/bash
# round-5 GPU call 9: the box kernel without the dead-direction spills (A/B
# on the driver's bench command, 20 and 200 frames)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05h
STEPS=200 LIBS="cur nospill" REPS=3 bash tools/ab_cmd.sh | tee gpurun_out/r05h/ab200.log
STEPS=20 LIBS="cur nospill" REPS=5 bash tools/ab_cmd.sh | tee gpurun_out/r05h/ab20.log
