#!/bin/bash
# A/B of output-invariant options on the BASELINE scenes (configs 3, 4, 5),
# after the wide-walk parity tests.  VARIANTS="a:opt15=0 b:opt15=1" tools/ab_fuse.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${VARIANTS:-"nofuse:opt15=0 fuse:opt15=1"}
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "wide or wavefront" --timeout 120 \
    --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo "parity rc=$?"; tail -20 gpurun_out/ab_parity.log; exit 1; }
  tail -1 gpurun_out/ab_parity.log
fi
timeout -k 10 200 python -u tools/ab_bench.py --scene sphere:6 --reps ${REPS:-5} $V > gpurun_out/ab_c3.log 2>&1 || { echo "c3 rc=$?"; tail -5 gpurun_out/ab_c3.log; exit 1; }
cat gpurun_out/ab_c3.log
if [ "${C4:-1}" = 1 ]; then
timeout -k 10 300 python -u tools/ab_bench.py --scene sphere:6 --w 3840 --h 2160 --spp 16 --reps ${REPS4:-2} $(for v in $V; do echo "$v,depth=8"; done) > gpurun_out/ab_c4.log 2>&1 || { echo "c4 rc=$?"; tail -5 gpurun_out/ab_c4.log; exit 1; }
cat gpurun_out/ab_c4.log
fi
timeout -k 10 300 python -u tools/ab_bench.py --scene random:10000000 --reps ${REPS:-5} $V > gpurun_out/ab_c5.log 2>&1 || { echo "c5 rc=$?"; tail -5 gpurun_out/ab_c5.log; exit 1; }
cat gpurun_out/ab_c5.log
