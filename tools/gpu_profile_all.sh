#!/bin/bash
# rocprofv3 evidence for every bench workload at the current source (TAG):
# tools/profile_workload.sh per workload; stops at the first failure.
#   TAG=r02s tools/gpu_profile_all.sh   (then, here: tools/summarize_all.sh r02s)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in ${WORKLOADS:-box sphere_1080p8 sphere_4k16_d8 synthetic10M_1080p8 synthetic10M_1080p8_exhaustive}; do
  WORKLOAD=$w bash tools/profile_workload.sh || { echo "profile $w failed"; exit 1; }
  echo "profiled $w"
done
