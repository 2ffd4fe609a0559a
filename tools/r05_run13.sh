#!/bin/bash
# round-5 GPU call 13: emulated 1/8 shares at (0,0,5): tail kernel on/off and
# 2 x 50 % against 3 x 33 %
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_group_parity.log 2>&1; rc=$?; tail -3 $OUT/pytest_group_parity.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for cfg in config5 config4; do
  for v in "3 33 0" "3 33 -1" "2 50 0" "2 50 -1"; do
    set -- $v
    CAM=reference GRID=$2 TAIL=$3 timeout -k 10 300 python3 tools/r04_scene_emu.py $cfg 8 $1 > $OUT/emu.log 2>&1 || { echo "emu $cfg $v rc=$?"; tail -5 $OUT/emu.log; exit 1; }
    grep '^{' $OUT/emu.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], d['contexts'], d['wf_grid_percent'], d['wf_tail'], d['full_frame_ms_median'], d['share_ms_median'], d['emulated_speedup'], d['shares_bitwise_equal'])" | tee -a $OUT/shares.log
  done
done
# the drop-in leg with members sharing this box's one GPU: both exchanges timed
for d in 0,0 0,0,0,0,0,0,0,0; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --no-scene-legs --no-cpu-baseline --group-devices $d > $OUT/group_$d.log 2>&1 || { echo "group $d rc=$?"; tail -5 $OUT/group_$d.log; exit 1; }
  grep '^{' $OUT/group_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d['group_leg']))" | tee -a $OUT/group.log
done
