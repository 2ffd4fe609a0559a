#!/bin/bash
# One library, option variants in one process (ab_bench alternates them):
#   SCENES="sphere:6 random:1000000" VARIANTS="a:opt13=1 b:opt13=2" tools/ab_opts.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sc in ${SCENES:-sphere:6}; do
  timeout -k 10 300 python3 tools/ab_bench.py --scene $sc --reps ${REPS:-3} ${AB_EXTRA:-} ${VARIANTS} > gpurun_out/ab_opts.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ab_opts.log; exit 1; }
  echo "$sc $(tail -1 gpurun_out/ab_opts.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["mean_ms"],2) for k,v in d["results"].items()})')"
done
