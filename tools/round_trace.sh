#!/bin/bash
# Per-dispatch durations of one emulated rank share (rocprofv3 kernel trace):
# the ray rounds of the wavefront pipeline, trace and shade per round.
#   EMU=8 SCENE=sphere W=1920 H=1080 SPP=8 DEPTH=4 tools/round_trace.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/rounds_${TAG:-x}
mkdir -p $OUT
PT_BENCH_EMULATE_RANKS=${EMU:-8} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 bench.py --scene ${SCENE:-sphere} --width ${W:-1920} --height ${H:-1080} --spp ${SPP:-8} --depth ${DEPTH:-4} \
  --steps 1 --warmup 1 --no-cpu-baseline --profile-run > $OUT/bench.log 2>&1 || { echo "rc=$?"; tail -20 $OUT/bench.log; exit 1; }
f=$(find $OUT -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if any(k in r["Kernel_Name"] for k in ("wf_trace", "wf_tail", "wf_shade", "wf_gen", "wf_fold"))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = len(rows) // 2   # the last frame
last = rows[n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:40]:40s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us")
PY
