#!/bin/bash
# round-5 GPU call 28: culled-item fill and frame assembly from host-computed
# item origins (no per-pixel tile arithmetic): the whole GPU suite and smoke
# on the product build, then the box on the driver's command against the
# previous build (ab/cur.so), the emulated root step, and two legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ze; mkdir -p $OUT
TAG=r05ze GATHER=0 BENCH=0 bash tools/r05_check.sh || exit $?
LIBS="cur fill" REPS=3 bash tools/ab_cmd.sh > $OUT/ab_box.log 2>&1 || { cat $OUT/ab_box.log; exit 1; }
cat $OUT/ab_box.log
for n in 8 4 2; do
  PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline > $OUT/emu$n.log 2>&1 || { echo "emu $n rc=$?"; tail -5 $OUT/emu$n.log; exit 1; }
  grep '^{' $OUT/emu$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d.get('host_issue_ms_per_step'))" | tee -a $OUT/emu_box.log
done
one() { # tag lib cam leg frames variant
  PTAMD_LIB=ab/$2.so CAM=$3 LEG="$4" FRAMES=$5 REPS=3 timeout -k 10 300 python3 tools/r05_leg_ab.py "$6" > $OUT/tmp.log 2>&1 || { echo "$1 $2 rc=$?"; tail -5 $OUT/tmp.log; exit 1; }
  grep "^rep" $OUT/tmp.log | sed "s/^/$1 $2 /" | tee -a $OUT/legs.log
}
for L in cur fill cur fill; do
  one c5ref $L reference "synthetic:10000000 1920 1080 8 4 1" 12 "g33@3:20=33" || exit 1
  one c3ref $L reference "sphere 1920 1080 8 4 3" 12 "g30@4:20=30" || exit 1
done
