#!/bin/bash
# wf_tail_kernel (PT_OPT_WF_TAIL): parity tests, then frame times of the
# large-scene configs at N=1 and as an emulated 1/8 share, per threshold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "tail_kernel" --timeout 200 \
  --timeout-method thread > gpurun_out/tail_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/tail_parity.log; exit 1; }
tail -1 gpurun_out/tail_parity.log
SPECS="sphere 1920 1080 8 4 3" VARIANTS="${V1:-17=0 17=1073741824 17=4000000 17=1000000 17=300000}" TAG=tail_a \
  timeout -k 10 600 tools/r03_scene_emu.sh || exit 1
SPECS="synthetic:10000000 1920 1080 8 4 3;sphere 3840 2160 16 8 2" VARIANTS="${V2:-17=0 17=1073741824 17=1000000}" \
  TAG=tail_b timeout -k 10 800 tools/r03_scene_emu.sh || exit 1
