#!/bin/bash
# round-5 GPU call 18 (no SLP vectorizer): rocprofv3 evidence of configs 4
# and 5, and the wide trace kernel's lane counters on config 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05t WORKLOADS="sphere_4k16_d8_refcam sphere_4k16_d8 synthetic10M_1080p8_refcam synthetic10M_1080p8 synthetic10M_1080p8_exhaustive" bash tools/r05_profile_all.sh
WTAG=r05t_wide bash tools/r05_wide_counters.sh
