#!/bin/bash
# WIDE_PAIR_LINES (PT_OPT_WIDE_BUILD 5): line-paired node order vs the SAH
# build's allocation order, same frames (parity checked between variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "wide_walk_matches_oracle and sah and 64" --timeout 200 \
  --timeout-method thread > gpurun_out/pair_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/pair_parity.log; exit 1; }
tail -1 gpurun_out/pair_parity.log
run() {
  local name=$1; shift
  timeout -k 10 500 python3 tools/ab_bench.py "$@" > gpurun_out/pair_$name.log 2>&1 \
    || { echo "$name rc=$?"; tail -5 gpurun_out/pair_$name.log; exit 1; }
  grep WARNING gpurun_out/pair_$name.log
  echo "$name $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pair_$name.log') if l.startswith('{')][-1]); print({k: round(v['mean_ms'],2) for k,v in d['results'].items()})")"
}
run c5 --scene random:10000000 --reps 4 sah:opt14=1 pair:opt14=5 sah2:opt14=1 pair2:opt14=5 || exit 1
run c3 --scene sphere:6 --reps 4 sah:opt14=1 pair:opt14=5 sah2:opt14=1 pair2:opt14=5 || exit 1
run c4 --scene sphere:6 --w 3840 --h 2160 --spp 16 --reps 2 sah:opt14=1,depth=8 pair:opt14=5,depth=8 || exit 1
