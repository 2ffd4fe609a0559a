#!/bin/bash
# SQ counters of the wavefront kernels (one rocprofv3 pass per group) for the
# sphere and the 10M cloud at the current source.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export GROUPS_LIST="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU
SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_SALU
GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
TAG=sq_sphere AB_ARGS="--scene sphere:6 v:" timeout -k 10 400 tools/wf_counters.sh > gpurun_out/sq_sphere.txt 2>&1 || { tail -5 gpurun_out/sq_sphere.txt; exit 1; }
TAG=sq_cloud AB_ARGS="--scene random:10000000 v:" timeout -k 10 500 tools/wf_counters.sh > gpurun_out/sq_cloud.txt 2>&1 || { tail -5 gpurun_out/sq_cloud.txt; exit 1; }
grep -h "wf_trace\|wf_tail" gpurun_out/sq_sphere.txt; echo; grep -h "wf_trace\|wf_tail" gpurun_out/sq_cloud.txt
