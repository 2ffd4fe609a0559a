#!/bin/bash
# round-5 GPU call 5: GPU tests, smoke, the driver's bench command, box lane
# counters, and rocprofv3 evidence of the box and config-3 workloads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05k GATHER=0 bash tools/r05_check.sh || exit $?
TAG=r05k_box bash tools/r05_box_counters.sh
TAG=r05q WORKLOADS="box sphere_1080p8_refcam sphere_1080p8" bash tools/r05_profile_all.sh
