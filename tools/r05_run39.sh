#!/bin/bash
# round-5 GPU call 39: the final tree -- the whole GPU suite and smoke, the
# driver's bench command twice (rooflines priced from profiles/r05zo at the
# same kernel SHA), a 200-frame box run, and the rocprofv3 kernel-trace stats
# of the driver's box command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zp; mkdir -p $OUT
TAG=r05zp GATHER=0 BENCH=0 bash tools/r05_check.sh || exit $?
for k in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench$k.log 2>&1 || { echo "bench $k rc=$?"; tail -5 $OUT/bench$k.log; exit 1; }
  grep '^{' $OUT/bench$k.log | cut -c1-300
done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline > $OUT/bench200.log 2>&1 || { echo "bench200 rc=$?"; exit 1; }
grep '^{' $OUT/bench200.log | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-scene-legs --no-cpu-baseline > $OUT/bench_rocprof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
grep '^{' $OUT/bench_rocprof.log | cut -c1-200
head -5 $OUT/prof/run_kernel_stats.csv
