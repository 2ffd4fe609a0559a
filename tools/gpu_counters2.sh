#!/bin/bash
# Counter groups (one rocprofv3 pass each) over one ab_bench configuration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctr2_${TAG:-x}
mkdir -p $OUT
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/ab_bench.py --no-parity --reps 1 ${AB_ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) rc=$?"; tail -5 $OUT/p$i.log; }
done <<< "$GROUPS_LIST"
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "render_kernel<false" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY
