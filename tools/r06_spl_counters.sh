#!/bin/bash
# round 6: SQ counters of the box render_kernel, one context, by sample lanes
# (20 frames + warm-up each; one --pmc pass per counter group)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06c}; mkdir -p $OUT
for spl in 1 4 8; do
  for grp in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_INSTS_LDS"; do
    n=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/spl${spl}_$n -o run -- \
      python3 tools/single_ctx.py 20 s$spl:2=$spl,8=0,9=0 > $OUT/spl${spl}_$n.log 2>&1 || { echo "pmc rc=$?"; tail $OUT/spl${spl}_$n.log; exit 1; }
  done
done

