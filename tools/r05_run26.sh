#!/bin/bash
# round-5 GPU call 26: the box root step of an emulated N-GPU run
# (PT_BENCH_EMULATE_RANKS) under sample lanes per pixel 1/2/4/8
# (PT_OPT_SAMPLE_LANES = 2) and item order (PT_OPT_ITEM_ORDER = 8), at the
# final build; the N > 1 default is lanes auto (8 at 8 spp), heaviest first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zc; mkdir -p $OUT
for n in 8 4 2; do
  for o in "2=8 8=1" "2=4 8=1" "2=2 8=1" "2=1 8=1" "2=4 8=0" "2=2 8=0"; do
    set -- $o
    tag="n${n}_$(echo $o | tr ' =' '_-')"
    PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline --opt $1 --opt $2 > $OUT/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 $OUT/$tag.log; exit 1; }
    grep '^{' $OUT/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', '$o', d['ms_per_step'], d.get('host_issue_ms_per_step'))" | tee -a $OUT/spl.log
  done
done
