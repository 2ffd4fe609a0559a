#!/bin/bash
# round 6: dump the measured mixed-lane schedule (PT_MIX_DUMP) and the frame times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06g}; mkdir -p $OUT
PT_MIX_DUMP=$OUT/sched.txt timeout -k 10 200 python tools/single_ctx.py 200 auto:9=0 m0:22=0,9=0 m50:22=50,9=0 > $OUT/single.log 2>&1 || { echo "rc=$?"; tail $OUT/single.log; exit 1; }
grep K= $OUT/single.log; head -1 $OUT/sched.txt
PTAMD_LIB=ab/wgtrace.so timeout -k 10 120 python tools/r06_wg_trace.py $OUT/auto.npz 9=1 > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail $OUT/trace.log; exit 1; }
head -4 $OUT/trace.log
