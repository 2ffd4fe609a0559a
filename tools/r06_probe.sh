#!/bin/bash
# round-6 GPU probe recipe: `tools/r06_probe.sh <tag> <cmd...>` runs one
# measurement command under a time limit, output to gpurun_out/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 ${PROBE_TIMEOUT:-300} "$@" > $OUT/out.log 2>&1
rc=$?
tail -40 $OUT/out.log
exit $rc
