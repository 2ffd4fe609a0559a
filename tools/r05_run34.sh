#!/bin/bash
# round-5 GPU call 34: live items' first pixels from the host as well
# (items_org: no tile arithmetic in the render kernel's prologue): parity
# and multi-rank GPU tests on the product build, then the box on the
# driver's command against the previous build (ab/fill.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zk; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_group.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
LIBS="fill org" REPS=4 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1 || { cat $OUT/ab_box.log; exit 1; }
cat $OUT/ab_box.log
