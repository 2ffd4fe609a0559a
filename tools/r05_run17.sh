#!/bin/bash
# round-5 GPU call 17 (device code built without the SLP vectorizer): GPU
# tests, smoke, box lane counters, rocprofv3 evidence of box and config 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05t GATHER=0 BENCH=0 bash tools/r05_check.sh || exit $?
TAG=r05t_box bash tools/r05_box_counters.sh
TAG=r05t WORKLOADS="box sphere_1080p8_refcam sphere_1080p8" bash tools/r05_profile_all.sh
