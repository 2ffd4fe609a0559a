#!/bin/bash
# rocprofv3 evidence for one bench workload, per MI355X_MICROARCH.md §HBM:
# a kernel-trace/stats pass, then FETCH_SIZE and WRITE_SIZE in passes of their
# own (they cannot share one on gfx950), plus VALU/SALU instruction counts,
# then tools/summarize_profile.py -> profiles/<TAG>/<WORKLOAD>_summary.json,
# which bench.py prices its roofline from (matched by kernel SHA and workload).
#   TAG=r02b WORKLOAD=box|sphere_1080p8[_refcam]|sphere_4k16_d8[_refcam]|synthetic10M_1080p8[_exhaustive|_refcam] tools/profile_workload.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-x}
WORKLOAD=${WORKLOAD:-box}
case $WORKLOAD in
  box) ARGS="--steps 20 --warmup 2"; STEPS=20; WARM=2 ;;
  sphere_1080p8) ARGS="--scene sphere --steps 2 --warmup 1"; STEPS=2; WARM=1 ;;
  synthetic10M_1080p8) ARGS="--scene synthetic:10000000 --steps 1 --warmup 1"; STEPS=1; WARM=1 ;;
  synthetic10M_1080p8_exhaustive) ARGS="--scene synthetic:10000000 --steps 1 --warmup 1 --opt 12=0"; STEPS=1; WARM=1 ;;
  sphere_4k16_d8) ARGS="--scene sphere --width 3840 --height 2160 --spp 16 --depth 8 --steps 1 --warmup 1"; STEPS=1; WARM=1 ;;
  # the legs' primary numbers: BASELINE's camera (0,0,5) (bench.py scene_leg)
  sphere_1080p8_refcam) ARGS="--scene sphere --camera reference --steps 2 --warmup 1"; STEPS=2; WARM=1 ;;
  sphere_4k16_d8_refcam) ARGS="--scene sphere --camera reference --width 3840 --height 2160 --spp 16 --depth 8 --steps 1 --warmup 1"; STEPS=1; WARM=1 ;;
  synthetic10M_1080p8_refcam) ARGS="--scene synthetic:10000000 --camera reference --steps 1 --warmup 1"; STEPS=1; WARM=1 ;;
  # the legs as bench.py times them (--leg: their contexts and traversal
  # grid, frames in flight; SCENE_LEGS): WARM = one frame per context
  sphere_1080p8_refcam_leg) ARGS="--leg config3 --leg-camera ref --steps 12"; STEPS=12; WARM=4 ;;
  sphere_1080p8_leg) ARGS="--leg config3 --leg-camera ff --steps 12"; STEPS=12; WARM=4 ;;
  sphere_4k16_d8_refcam_leg) ARGS="--leg config4 --leg-camera ref --steps 6"; STEPS=6; WARM=2 ;;
  sphere_4k16_d8_leg) ARGS="--leg config4 --leg-camera ff --steps 6"; STEPS=6; WARM=2 ;;
  synthetic10M_1080p8_refcam_leg) ARGS="--leg config5 --leg-camera ref --steps 12"; STEPS=12; WARM=3 ;;
  synthetic10M_1080p8_leg) ARGS="--leg config5 --leg-camera ff --steps 12"; STEPS=12; WARM=2 ;;
  *) echo "unknown WORKLOAD $WORKLOAD"; exit 2 ;;
esac
OUT=gpurun_out/prof_${TAG}_${WORKLOAD}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $ARGS --profile-run > $OUT/bench_trace.log 2>&1 \
  || { echo "trace rc=$?"; tail -20 $OUT/bench_trace.log; exit 1; }
grep '^{' $OUT/bench_trace.log | tail -1 | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum"; do
  n=${c%% *}
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$n -o run -- \
    python3 bench.py $ARGS --profile-run > $OUT/bench_$n.log 2>&1 \
    || { echo "pmc $c rc=$?"; tail -20 $OUT/bench_$n.log; exit 1; }
done
echo "frames=$((STEPS + WARM))" > $OUT/frames.txt
# summarize in the container (profiles/ written on the box does not come back):
#   python3 tools/summarize_profile.py $TAG $WORKLOAD $((STEPS + WARM))
