#!/bin/bash
# round 6: the headline's launch events (--timing-every 0: none) and three
# contexts in flight (--streams 3), against the default, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06p}; mkdir -p $OUT
one() { name=$1; shift; timeout -k 10 200 python bench.py --no-scene-legs --no-cpu-baseline "$@" > $OUT/$name.log 2>&1 || { echo "$name rc=$?"; tail $OUT/$name.log; exit 1; }; echo "$name $(tail -1 $OUT/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("verified_vs_oracle"))')"; }
for rep in 1 2; do
  one base200_$rep --steps 200 --warmup 10
  one t0_200_$rep --steps 200 --warmup 10 --timing-every 0
  one s3_200_$rep --steps 200 --warmup 10 --streams 3
  one base20_$rep --steps 20 --warmup 5
  one t0_20_$rep --steps 20 --warmup 5 --timing-every 0
  one s3_20_$rep --steps 20 --warmup 5 --streams 3
done
