#!/bin/bash
# Emulated root step (native loop) per N under kernel options: sample lanes
# (2=) and item order (8=), one run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/share_opts
mkdir -p $OUT
declare -A OPTS
OPTS[2]=${OPTS2:-'|2=1 8=0|2=2 8=0|2=4 8=0|2=1|2=2'}
OPTS[4]=${OPTS4:-'|2=1 8=0|2=2 8=0|2=4 8=0|2=1|2=2'}
OPTS[8]=${OPTS8:-'|2=1 8=0|2=2 8=0|2=4 8=0|2=1|2=2'}
for rep in $(seq ${REPS:-1}); do
for n in ${NS:-2 4 8}; do
  IFS='|' read -ra LIST <<< "${OPTS[$n]}"
  for o in "${LIST[@]}"; do
    args=""; for kv in $o; do args="$args --opt $kv"; done
    tag=$(echo "n${n}_${o}_$rep" | tr ' =' '_-')
    PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-scene-legs --steps 400 $args \
      > $OUT/$tag.log 2>&1 || { echo "rc=$? $tag"; tail -5 $OUT/$tag.log; exit 1; }
    echo "n=$n opts=[$o] $(grep '^{' $OUT/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
done
