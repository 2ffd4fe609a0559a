#!/bin/bash
# A/B of pt_set_option variants on the BASELINE device-memory scenes (one process per scene):
#   AB_VARIANTS="a:opt14=0 b:opt14=1" AB_SCENES="sphere:6 random:10000000" tools/ab_scenes2.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for S in ${AB_SCENES:-sphere:6 random:10000000}; do
  n=${S//:/_}
  timeout -k 10 ${AB_TIMEOUT:-300} python3 tools/ab_bench.py --scene $S --reps ${AB_REPS:-3} ${AB_ARGS:-} ${AB_VARIANTS} > gpurun_out/ab2_$n.log 2>&1 || { echo "$S rc=$?"; tail -5 gpurun_out/ab2_$n.log; exit 1; }
  grep -v '^{' gpurun_out/ab2_$n.log | tail -3
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab2_$n.log') if l.startswith('{')][-1]); print('$S', {k: round(v['mean_ms'],2) for k,v in d['results'].items()})"
done
