#!/bin/bash
# HBM traffic of the large-scene path: rocprofv3
# kernel trace + separate FETCH_SIZE and WRITE_SIZE passes over a short bench
# of each scene.  SCENES entries: scene:spp:steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for spec in ${SCENES:-"sphere:8:2" "synthetic:10000000:1:1"}; do
  IFS=: read -r a b c d <<< "$spec"
  if [ "$a" = "synthetic" ]; then scene="$a:$b"; spp=$c; steps=$d; else scene=$a; spp=$b; steps=$c; fi
  tag=$(echo $scene | tr ':' '_')
  OUT=gpurun_out/sprof_${TAG:-x}_$tag
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --scene $scene --spp $spp --steps $steps --warmup 1 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 \
    || { echo "$scene trace rc=$?"; tail -20 $OUT/bench_trace.log; exit 1; }
  grep '^{' $OUT/bench_trace.log | tail -1 | cut -c1-400
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
      python3 bench.py --scene $scene --spp $spp --steps $steps --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 \
      || { echo "$scene pmc $c rc=$?"; tail -20 $OUT/bench_$c.log; exit 1; }
  done
  echo "$scene done"
done
