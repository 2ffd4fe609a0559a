#!/bin/bash
# round 6: one-GPU emulations of the N-GPU runs at the round-6 build -- the
# box root step (native loop, culled items assembled once per buffer) at
# N = 2/4/8, three runs each, N = 1 beside them; configs 4 and 5 rank-0 1/8
# shares at (0,0,5) as dist_scene_leg runs them (3 contexts at 33 %)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06n}; mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline --compare-no-cull 1 > $OUT/n1_$rep.log 2>&1 || { echo "n1 rc=$?"; tail $OUT/n1_$rep.log; exit 1; }
  echo "N=1 $(tail -1 $OUT/n1_$rep.log | cut -c1-200 | grep -o '"ms_per_step":[0-9.]*')"
  for n in 2 4 8; do
    PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-scene-legs > $OUT/emu${n}_$rep.log 2>&1 || { echo "emu$n rc=$?"; tail $OUT/emu${n}_$rep.log; exit 1; }
    echo "N=$n $(tail -1 $OUT/emu${n}_$rep.log | grep -o '"ms_per_step":[0-9.]*')"
  done
done
for cfg in config4 config5; do
  CAM=reference GRID=33 timeout -k 10 400 python tools/r04_scene_emu.py $cfg 8 3 > $OUT/scene_$cfg.log 2>&1 || { echo "$cfg rc=$?"; tail $OUT/scene_$cfg.log; exit 1; }
  tail -1 $OUT/scene_$cfg.log | cut -c1-400
done
