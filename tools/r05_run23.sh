#!/bin/bash
# round-5 GPU call 23: the one-GPU emulations of the N-GPU runs at the no-SLP
# build -- the box root step at N = 2/4/8 (PT_BENCH_EMULATE_RANKS) and rank
# 0's 1/8 share of configs 4/5 on 3 contexts at 33 % (the dist legs' setting)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05y; mkdir -p $OUT
for n in 1 2 4 8; do
  PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline > $OUT/emu$n.log 2>&1 || { echo "emu $n rc=$?"; tail -5 $OUT/emu$n.log; exit 1; }
  grep '^{' $OUT/emu$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d.get('host_issue_ms_per_step'))" | tee -a $OUT/emu_box.log
done
for cfg in config4 config5; do
  CAM=reference GRID=33 TAIL=0 timeout -k 10 300 python3 tools/r04_scene_emu.py $cfg 8 3 12 > $OUT/emu_$cfg.log 2>&1 || { echo "emu $cfg rc=$?"; tail -5 $OUT/emu_$cfg.log; exit 1; }
  grep '^{' $OUT/emu_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['contexts'], d['wf_grid_percent'], d['full_frame_ms_median'], d['share_ms_median'], d['emulated_speedup'], d['shares_bitwise_equal'])" | tee -a $OUT/shares.log
done
