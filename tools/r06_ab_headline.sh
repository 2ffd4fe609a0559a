#!/bin/bash
# round 6: the headline (two contexts in flight) with the measured whole-tile
# order (PT_OPT_MIXED_LANES -1, the default) against uniform scan order (22=0),
# 200-frame and the driver's 20-frame runs, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06m}; mkdir -p $OUT
one() { name=$1; shift; timeout -k 10 200 python bench.py --no-scene-legs --no-cpu-baseline "$@" > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail $OUT/$name.log; exit 1; }; echo "$name $(tail -1 $OUT/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("lane_schedule"), d.get("single_context",{}).get("ms_per_step"))')"; }
for rep in 1 2; do
  one meas200_$rep --steps 200 --warmup 10
  one off200_$rep --steps 200 --warmup 10 --opt 22=0
  one meas20_$rep --steps 20 --warmup 5
  one off20_$rep --steps 20 --warmup 5 --opt 22=0
done
