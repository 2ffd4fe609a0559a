#!/bin/bash
# Run a command while appending a timestamp to gpurun_out/heartbeat.txt every
# 60 s, for GPU steps that print nothing for minutes (a 10M-triangle profile
# pass under rocprofv3); the command keeps its own time limits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
(while sleep 60; do date >> gpurun_out/heartbeat.txt; done) &
hb=$!
"$@"
rc=$?
kill $hb
exit $rc
