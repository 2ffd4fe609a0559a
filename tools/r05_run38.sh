#!/bin/bash
# round-5 GPU call 38: rocprofv3 evidence of all eight workloads at the final
# kernel build (the final kernel sources), box and wide-kernel counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05zo_box bash tools/r05_box_counters.sh
TAG=r05zo bash tools/r05_profile_all.sh || exit 1
WTAG=r05zo_wide bash tools/r05_wide_counters.sh
