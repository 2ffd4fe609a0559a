#!/bin/bash
# round 6: per-workgroup timelines of the box frame (probe build ab/wgtrace.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06e}; mkdir -p $OUT
for v in "m0:22=0,8=0,9=1" "m50:22=50,8=0" "m100:22=100,8=0" "s1:2=1,22=0,8=0" "s4o1:22=0,8=1"; do
  name=${v%%:*}; opts=${v#*:}
  PTAMD_LIB=ab/wgtrace.so timeout -k 10 120 python tools/r06_wg_trace.py $OUT/$name.npz $opts > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail $OUT/$name.log; exit 1; }
  cat $OUT/$name.log | grep -v amdgpu.ids
done
