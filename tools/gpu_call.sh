#!/bin/bash
# One GPU call, assembled from named steps (replaces round 5's forty one-off
# tools/r05_run*.sh recipes; they stay in the git history, commit 2cc4b50).
#
#   TAG=r06x tools/gpu_call.sh STEP [STEP ...]
#
# Every step writes under gpurun_out/$TAG/, runs under its own time limit and
# the call stops at the first failing step (no GPU step after a fault, abort
# or timeout).  Steps:
#   tests             the whole GPU suite (pytest -m gpu)
#   tests:EXPR        GPU tests matching -k EXPR
#   smoke             __graft_entry__.smoke()
#   bench             the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench_default     bench.py with no flags (200 steps, legs, CPU baseline)
#   bench200          the box alone, 200 steps (no legs, no CPU baseline)
#   single[:K]        tools/single_ctx.py K (default 200): the one-context drop-in frame
#   emu:N             rank 0 of an emulated N-GPU box run (PT_BENCH_EMULATE_RANKS=N, 200 steps)
#   profile:WORKLOAD  tools/profile_workload.sh for WORKLOAD (rocprofv3 trace + PMC passes)
#   rocprof_bench     the driver's command under rocprofv3 --kernel-trace --stats
#   counters:box      SQ counters of the box render_kernel at the bench's options
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {   # run LIMIT LOG CMD...: one GPU step under its own limit
  local limit=$1 log=$2
  shift 2
  timeout -k 10 "$limit" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step failed (rc=$rc): $*"
    tail -30 "$log"
    exit $rc
  fi
}

for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      run 600 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread
      tail -3 "$OUT/pytest_gpu.log" ;;
    tests:*)
      run 600 "$OUT/pytest_${step#tests:}.log" python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread -k "${step#tests:}"
      tail -3 "$OUT/pytest_${step#tests:}.log" ;;
    smoke)
      run 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 "$OUT/smoke.log" ;;
    bench)
      PT_BENCH_DETAIL=$OUT/bench_detail.json run 600 "$OUT/bench.log" python bench.py --gpus 1 --steps 20 --warmup 5
      tail -1 "$OUT/bench.log" | cut -c1-600 ;;
    bench_default)
      PT_BENCH_DETAIL=$OUT/bench_default_detail.json run 600 "$OUT/bench_default.log" python bench.py
      tail -1 "$OUT/bench_default.log" | cut -c1-600 ;;
    bench200)
      PT_BENCH_DETAIL=$OUT/bench200_detail.json run 300 "$OUT/bench200.log" python bench.py --steps 200 \
        --no-scene-legs --no-cpu-baseline
      tail -1 "$OUT/bench200.log" | cut -c1-400 ;;
    single|single:*)
      k=${step#single}; k=${k#:}
      run 300 "$OUT/single.log" python tools/single_ctx.py "${k:-200}" default: timing_off:9=0
      grep K= "$OUT/single.log" ;;
    emu:*)
      n=${step#emu:}
      PT_BENCH_EMULATE_RANKS=$n PT_BENCH_DETAIL=$OUT/emu$n.json run 300 "$OUT/emu$n.log" python bench.py --steps 200 \
        --warmup 10 --no-scene-legs
      tail -1 "$OUT/emu$n.log" | cut -c1-300 ;;
    profile:*)
      TAG=$TAG WORKLOAD=${step#profile:} run 1100 "$OUT/profile_${step#profile:}.log" tools/profile_workload.sh
      tail -3 "$OUT/profile_${step#profile:}.log" ;;
    rocprof_bench)
      run 900 "$OUT/bench_rocprof.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" \
        -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
      tail -1 "$OUT/bench_rocprof.log" | cut -c1-300 ;;
    counters:box)
      run 300 "$OUT/box_counters.log" tools/r05_box_counters.sh
      tail -5 "$OUT/box_counters.log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
