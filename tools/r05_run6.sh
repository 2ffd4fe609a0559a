#!/bin/bash
# round-5 GPU call 6: rocprofv3 evidence of the config-4 and config-5 workloads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05q WORKLOADS="sphere_4k16_d8_refcam sphere_4k16_d8 synthetic10M_1080p8_refcam synthetic10M_1080p8 synthetic10M_1080p8_exhaustive" bash tools/r05_profile_all.sh
WTAG=r05x bash tools/r05_wide_counters.sh
