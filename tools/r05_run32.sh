#!/bin/bash
# round-5 GPU call 32: the box's item order on the driver's 20-frame command
# and over 200 frames at the final build: scan order (the bench's default,
# PT_OPT_ITEM_ORDER 0) against heaviest first (1), alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zi; mkdir -p $OUT
for st in 20 200; do
  for i in 1 2 3; do
    for o in 0 1; do
      timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --no-scene-legs --no-cpu-baseline --opt 8=$o > $OUT/o${o}_s${st}_$i.log 2>&1 || { echo "o$o rc=$?"; tail -5 $OUT/o${o}_s${st}_$i.log; exit 1; }
      grep '^{' $OUT/o${o}_s${st}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps $st order $o', d['ms_per_step'])" | tee -a $OUT/order.log
    done
  done
done
