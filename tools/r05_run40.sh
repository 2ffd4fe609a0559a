#!/bin/bash
# round-5 GPU call 40: bench.py with no flags (N = 1, 200 steps, 10 warmup,
# scene legs and CPU baseline) on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zq; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_default.log; exit 1; }
grep '^{' $OUT/bench_default.log | cut -c1-300
