#!/bin/bash
# Bench lines for the other BASELINE configs: sphere (Sylveon substitute),
# synthetic clouds (1M, 10M triangles) — 1 GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in ${SCENES:-"sphere:8:3" "synthetic:1000000:1:2" "synthetic:10000000:1:1"}; do
  IFS=: read -r name arg spp steps <<< "$spec"
  scene=$name; [ "$name" = "synthetic" ] && scene="synthetic:$arg" && spp=${spp}; [ "$name" = "sphere" ] && spp=$arg && steps=$spp
  tag=$(echo $scene | tr ':' '_')
  timeout -k 10 600 python bench.py --scene $scene --spp ${spp} --steps ${steps:-3} --warmup 1 --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo "$scene rc=$?"; tail -20 gpurun_out/bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/bench_$tag.log | tail -1
done
