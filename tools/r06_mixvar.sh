#!/bin/bash
# round 6: measured mixed-lane schedule, tail fraction at 4 lanes (PT_MIX_TAIL4, tuning), one process each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06i}; mkdir -p $OUT
run() { name=$1; shift; env "$@" timeout -k 10 120 python tools/single_ctx.py 200 $name: > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail $OUT/$name.log; exit 1; }; grep K= $OUT/$name.log; }
run lpt2 X=1
run tail05 PT_MIX_TAIL4=0.05
run tail10 PT_MIX_TAIL4=0.1
run tail20 PT_MIX_TAIL4=0.2
run lpt2b X=1
run tail35 PT_MIX_TAIL4=0.35
timeout -k 10 120 python tools/single_ctx.py 200 m50:22=50 m0:22=0 > $OUT/static.log 2>&1; grep K= $OUT/static.log
