#!/bin/bash
# PT_OPT_WF_TAIL thresholds (small: the tail kernel takes only the last
# rounds) on the large-scene configs, whole frames and emulated 1/8 shares.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${THRS:-0 50000 150000 400000}
run() {   # name, ab_bench args..., extra variant keys
  local name=$1; shift; local extra=$1; shift
  local vs=""; for t in $T; do vs="$vs t$t:opt17=$t$extra"; done
  timeout -k 10 500 python3 tools/ab_bench.py "$@" --reps ${REPS:-3} $vs > gpurun_out/thr_$name.log 2>&1 \
    || { echo "$name rc=$?"; tail -5 gpurun_out/thr_$name.log; exit 1; }
  echo "$name $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/thr_$name.log') if l.startswith('{')][-1]); print({k: round(v['mean_ms'],2) for k,v in d['results'].items()})")"
}
run c4_n8 ",depth=8,nr=8" --scene sphere:6 --w 3840 --h 2160 --spp 16 || exit 1
run c5_n8 ",nr=8" --scene random:10000000 || exit 1
run c3_n8 ",nr=8" --scene sphere:6 || exit 1
run c3_n1 "" --scene sphere:6 || exit 1
run c5_n1 "" --scene random:10000000 || exit 1
REPS=2 run c4_n1 ",depth=8" --scene sphere:6 --w 3840 --h 2160 --spp 16 || exit 1
