#!/bin/bash
# PMC counter passes over the A/B bench (render kernel); one pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr_${TAG:-x}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/ab_bench.py --reps 2 ${AB_ARGS:-v:lds=1} > $OUT/p$i.log 2>&1 || echo "pass $i ($grp) rc=$?"
done
ls $OUT
