#!/bin/bash
# Per-kernel time split of one scene frame (rocprofv3 kernel trace + stats):
#   AB_SCENES="sphere:6 random:10000000" tools/gpu_split.sh   [PTAMD_LIB=ab/x.so]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for S in ${AB_SCENES:-sphere:6 random:10000000}; do
  n=${S//:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split_$n -o run -- \
    python3 tools/ab_bench.py --scene $S --reps ${AB_REPS:-2} v: > gpurun_out/split_$n.log 2>&1 || { echo "$S rc=$?"; tail -5 gpurun_out/split_$n.log; exit 1; }
  echo "== $S"; cut -d, -f1-4 gpurun_out/split_$n/run_kernel_stats.csv | head -8
done
