#!/bin/bash
# GPU-box profile: kernel trace + stats of the bench, then HBM counters in
# separate passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
STEPS=${STEPS:-20}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $OUT/bench_trace.log; exit 1; }
tail -2 $OUT/bench_trace.log
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
  n=${c%% *}
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$n -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$n.log 2>&1 || { echo "pmc $c rc=$?"; tail -20 $OUT/bench_$n.log; exit 1; }
done
find $OUT -name '*.csv' | head -20
