#!/bin/bash
# Flush-window use of the wide trace kernel at the legs' settings (PT_WIDE_PROBE_FLUSH build ab/fprobe.so).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for args in "--scene sphere:6 --refcam --grid 30" "--scene sphere:6 --grid 100" "--scene random:10000000 --refcam --grid 33"; do
  PTAMD_LIB=ab/fprobe.so timeout -k 10 200 python3 tools/flush_probe.py $args | tail -1
done
