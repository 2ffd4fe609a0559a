#!/bin/bash
# round-5 GPU call 35: rocprofv3 evidence of all eight workloads at the final
# kernel build (live and culled item origins from the host), box and wide-kernel counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05zl_box bash tools/r05_box_counters.sh
TAG=r05zl bash tools/r05_profile_all.sh || exit 1
WTAG=r05zl_wide bash tools/r05_wide_counters.sh
