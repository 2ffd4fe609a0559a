#!/bin/bash
# round 6: box 1080p8 per-sample cost by sample lanes -- one context (the
# drop-in frame, launch timing off, scan order) and two contexts in flight
# (bench.py's headline setup), 200 frames each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06b}; mkdir -p $OUT
timeout -k 10 200 python tools/single_ctx.py 200 s4:2=4,8=0,9=0 s1:2=1,8=0,9=0 s2:2=2,8=0,9=0 s8:2=8,8=0,9=0 s4o1:2=4,8=1,9=0 > $OUT/single.log 2>&1 || { echo "single rc=$?"; tail $OUT/single.log; exit 1; }
cat $OUT/single.log | grep K=
for spl in 1 2 4 8; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline --compare-no-cull 0 --opt 2=$spl --opt 8=0 > $OUT/pipe_spl$spl.log 2>&1 || { echo "pipe rc=$?"; tail $OUT/pipe_spl$spl.log; exit 1; }
  echo "pipelined spl$spl: $(tail -1 $OUT/pipe_spl$spl.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("single_context",{}).get("ms_per_step"))')"
done
