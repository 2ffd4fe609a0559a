#!/bin/bash
# 8-wide nodes vs 64-B 4-wide nodes: wide-walk parity tests (every layout),
# then A/B frames on the BASELINE scenes (configs 3, 4, 5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "wide_walk_matches_oracle" --timeout 120 \
  --timeout-method thread > gpurun_out/w8_parity.log 2>&1 || { echo "parity rc=$?"; tail -30 gpurun_out/w8_parity.log; exit 1; }
tail -1 gpurun_out/w8_parity.log
V=${VARIANTS:-"n64:opt16=64 n80:opt16=80"}
timeout -k 10 200 python -u tools/ab_bench.py --scene sphere:6 --reps ${REPS:-5} $V > gpurun_out/w8_c3.log 2>&1 || { echo "c3 rc=$?"; tail -5 gpurun_out/w8_c3.log; exit 1; }
tail -3 gpurun_out/w8_c3.log
timeout -k 10 300 python -u tools/ab_bench.py --scene random:10000000 --reps ${REPS:-5} $V > gpurun_out/w8_c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 gpurun_out/w8_c5.log; exit 1; }
tail -3 gpurun_out/w8_c5.log
timeout -k 10 300 python -u tools/ab_bench.py --scene sphere:6 --w 3840 --h 2160 --spp 16 --reps 2 $(for v in $V; do echo "$v,depth=8"; done) > gpurun_out/w8_c4.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/w8_c4.log; exit 1; }
tail -3 gpurun_out/w8_c4.log
