#!/bin/bash
# Parity subset of the wavefront / wide-walk GPU tests on the in-tree library,
# then an A/B of ab/<lib>.so builds on the BASELINE scenes (configs 3 and 5).
#   LIBS="base new" tools/ab_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "${PARITY_K:-wide or wavefront}" --timeout 120 \
  --timeout-method thread > gpurun_out/abc_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/abc_parity.log; exit 1; }
tail -1 gpurun_out/abc_parity.log
AB_SCENES=${AB_SCENES:-"sphere:6 random:10000000"} AB_ITERS=${AB_ITERS:-2} timeout -k 10 800 tools/ab_libs_scenes.sh
