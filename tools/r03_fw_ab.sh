#!/bin/bash
# PT_WIDE_FLUSH_WAVE A/B: wide-walk and tail parity on the new build, then
# library builds fw0 (per-lane flush) / fw1 (wave-wide flush) alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PTAMD_LIB=ab/fw1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q \
  -k "wide or wavefront or tail or config" --timeout 200 --timeout-method thread > gpurun_out/fw_parity.log 2>&1 \
  || { echo "parity rc=$?"; tail -30 gpurun_out/fw_parity.log; exit 1; }
tail -1 gpurun_out/fw_parity.log
LIBS="fw0 fw1" AB_SCENES="sphere:6 random:10000000" AB_ITERS=2 AB_REPS=3 timeout -k 10 700 tools/ab_libs_scenes.sh || exit 1
