#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at the first GPU
# fault / abort / timeout (exit codes other than 0 or 1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-420} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 > gpurun_out/bench.log 2>&1
brc=$?
cat gpurun_out/bench.log | tail -5
exit $brc
