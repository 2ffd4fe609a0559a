#!/bin/bash
# Counter groups (one rocprofv3 pass each) over one ab_bench frame, reported
# per kernel family (sums over dispatches / frames).  GROUPS_LIST: one
# counter group per line.  AB_ARGS: ab_bench arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/wfc_${TAG:-x}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 tools/ab_bench.py --no-parity --reps 1 ${AB_ARGS} > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/ab_bench.py --no-parity --reps 1 ${AB_ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done <<< "$GROUPS_LIST"
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
fam = lambda n: next((k for k in ("wf_trace", "wf_tail", "wf_shade", "wf_gen", "wf_fold", "render_kernel") if k in n), None)
agg = collections.defaultdict(float)
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = fam(r["Kernel_Name"])
        if k:
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print(f"{k:14s} {c:32s} {v:.6g}")
for r in csv.DictReader(open(glob.glob(out + "/trace/run_kernel_stats.csv")[0])):
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} total_ms {float(r['TotalDurationNs'])/1e6:9.2f}")
PY
