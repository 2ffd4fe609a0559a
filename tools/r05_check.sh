#!/bin/bash
# Round-5 GPU check: GPU tests, smoke, the gather ceilings at the trace
# kernel's memory-level parallelism, then the driver's bench command.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05a}
mkdir -p $OUT
stop() { echo "$1 rc=$2: stopping"; exit $2; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && stop pytest $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || stop smoke $?
  cat $OUT/smoke.log
fi
if [ "${GATHER:-1}" = "1" ]; then
  timeout -k 10 120 tools/gather_roof mlp > $OUT/gather_roof_mlp.jsonl 2>&1 || stop gather_roof $?
  cat $OUT/gather_roof_mlp.jsonl
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || stop bench $?
  grep '^{' $OUT/bench.log | cut -c1-400
fi
