#!/bin/bash
# round 6: mixed sample lanes -- parity tests, then the single-context sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06f}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "mixed or sample_lanes or box_1080p or box_matches" > $OUT/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python tools/single_ctx.py 200 auto:9=0 m0:22=0,9=0,8=0 m50:22=50,9=0,8=0 autoo0:9=0,8=0 autot1: > $OUT/single.log 2>&1 || { echo "single rc=$?"; tail $OUT/single.log; exit 1; }
grep K= $OUT/single.log
