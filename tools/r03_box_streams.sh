#!/bin/bash
# Box headline: contexts in flight (--streams) x sample lanes, one run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/box_streams
mkdir -p $OUT
for rep in 1 2; do
for st in 2 3 4; do
  for o in "" "--opt 2=2"; do
    tag=st${st}_$(echo "$o" | tr ' =' '_-')_$rep
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-scene-legs --streams $st $o > $OUT/$tag.log 2>&1 \
      || { echo "rc=$? $tag"; tail -5 $OUT/$tag.log; exit 1; }
    echo "streams=$st [$o] $(grep '^{' $OUT/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
done
