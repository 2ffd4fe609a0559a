#!/bin/bash
# SQ counters of the box render_kernel at the bench's options (one lane per
# pixel, items in scan order): lanes per VALU instruction, wait and issue
# buckets, LDS cycles.  Output: gpurun_out/<TAG>_counters.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05box}
export TAG
export AB_ARGS="--reps 2 b:opt2=1,opt8=0,opt3=1"
export GROUPS_LIST="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES
SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
bash tools/wf_counters.sh > gpurun_out/${TAG}_counters.txt 2>&1
echo rc=$?
