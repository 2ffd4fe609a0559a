#!/bin/bash
# One PMC pass per (variant, group): SQ instruction/utilisation counters of the
# render kernel for each ab_bench variant given in VARIANTS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ctrv_${TAG:-x}
mkdir -p $OUT
for v in ${VARIANTS}; do
  n=${v%%:*}
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS \
    --output-format csv -d $OUT/$n -o run -- python3 tools/ab_bench.py --no-parity --reps 2 $v > $OUT/$n.log 2>&1 || { echo "variant $n rc=$?"; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
for d in sorted(glob.glob(out + "/*/")):
    f = glob.glob(d + "run_counter_collection.csv")
    if not f:
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "render_kernel<false" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    util = m["SQ_THREAD_CYCLES_VALU"] / (m["SQ_ACTIVE_INST_VALU"] * 64) if m.get("SQ_ACTIVE_INST_VALU") else 0
    print(os.path.basename(d.rstrip("/")), {k: int(v) for k, v in m.items()}, "lane_util=%.3f" % util)
PY
