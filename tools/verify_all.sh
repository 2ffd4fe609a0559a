#!/bin/bash
# Round-end style check on one GPU box: every -m gpu test, smoke(), then the
# default bench line.  Each step has its own time limit; the first failure
# (or fault / abort / timeout) ends the script.
#   TAG=r03b tools/verify_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-x}
OUT=gpurun_out/verify_$TAG
mkdir -p $OUT
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit 0; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 \
  || { echo "bench rc=$?"; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | cut -c1-400
