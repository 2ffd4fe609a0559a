#!/bin/bash
# Quick check of a kernel change on the headline: smoke, the LDS-path parity
# tests, then the default box bench line twice (no scene legs).
#   PYK=... (pytest -k), EXTRA=... (bench args), REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick_${TAG:-x}
mkdir -p $OUT
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${PYK:-box or lds or grid or edge or random or shadow_skip or sample_lanes or culling}" > $OUT/parity.log 2>&1 \
  || { echo "pytest rc=$?"; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
for rep in $(seq ${REPS:-2}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline ${EXTRA:---no-scene-legs} > $OUT/bench_$rep.log 2>&1 \
    || { echo "bench rc=$?"; tail -5 $OUT/bench_$rep.log; exit 1; }
  grep '^{' $OUT/bench_$rep.log | python3 -c '
import json,sys
d=json.loads(sys.stdin.read())
print("box", d["value"], d["ms_per_step"])
for k,v in d.get("configs",{}).items(): print(k, v["ms_per_step"], v["reference_camera"]["ms_per_step"])'
done
