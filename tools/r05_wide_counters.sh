#!/bin/bash
# SQ counters of the wavefront kernels on the config-3 frame (1080p 8 spp,
# the level-6 sphere) at BASELINE's camera: a full traversal grid against the
# leg's 25 % (more rays per lane per round): lanes per VALU instruction and
# wait buckets of wf_trace_wide_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GROUPS_LIST="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
for g in ${GRIDS:-100 25}; do
  CAM=reference TAG=${WTAG:-r05w}_g$g AB_ARGS="--scene sphere:6 --reps 1 v:opt20=$g" bash tools/wf_counters.sh > gpurun_out/${WTAG:-r05w}_g${g}.txt 2>&1
  grep wf_trace gpurun_out/${WTAG:-r05w}_g${g}.txt
done
