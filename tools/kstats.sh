#!/bin/bash
# Per-kernel time split of bench workloads (rocprofv3 kernel trace + stats only):
#   WORKLOADS="sphere_1080p8 synthetic10M_1080p8" TAG=x tools/kstats.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for W in ${WORKLOADS:-sphere_1080p8}; do
  case $W in
    box) ARGS="--steps 20 --warmup 2" ;;
    sphere_1080p8) ARGS="--scene sphere --steps 2 --warmup 1" ;;
    synthetic10M_1080p8) ARGS="--scene synthetic:10000000 --steps 1 --warmup 1" ;;
    sphere_4k16_d8) ARGS="--scene sphere --width 3840 --height 2160 --spp 16 --depth 8 --steps 1 --warmup 1" ;;
    *) echo "unknown $W"; exit 2 ;;
  esac
  OUT=gpurun_out/kstats_${TAG:-x}_$W
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py $ARGS ${EXTRA:-} --profile-run > $OUT/bench.log 2>&1 || { echo "$W rc=$?"; tail -20 $OUT/bench.log; exit 1; }
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  echo "== $W"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:6]: print(r['Name'][:70], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), 'ms total', r['Percentage'])
"
done
