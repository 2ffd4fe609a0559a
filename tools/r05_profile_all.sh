#!/bin/bash
# rocprofv3 evidence for every bench workload at the current kernel source
# (WORKLOADS overrides the list), TAG names the profiles/ directory.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG=${TAG:-r05p}
for w in ${WORKLOADS:-box sphere_1080p8_refcam sphere_1080p8 sphere_4k16_d8_refcam sphere_4k16_d8 synthetic10M_1080p8_refcam synthetic10M_1080p8 synthetic10M_1080p8_exhaustive}; do
  echo "== $w"
  WORKLOAD=$w bash tools/profile_workload.sh || { echo "profile $w failed"; exit 1; }
done
