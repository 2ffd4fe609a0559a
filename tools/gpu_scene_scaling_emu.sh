#!/bin/bash
# 1-GPU box: rank 0's step of an N-GPU tile split (PT_BENCH_EMULATE_RANKS)
# for the large-scene configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/scene_emu_${TAG:-x}.jsonl
: > $OUT
# SPECS: ';'-separated "scene width height spp depth steps" entries
IFS=';' read -ra specs <<< "${SPECS:-sphere 3840 2160 16 8 1;synthetic:10000000 1920 1080 1 4 1}"
for spec in "${specs[@]}"; do
  read -r scene w h spp depth steps <<< "$spec"
  for n in ${RANKS:-1 8}; do
    log=gpurun_out/scene_emu_$(echo $scene | tr ':' '_')_n$n.log
    PT_BENCH_EMULATE_RANKS=$n timeout -k 10 500 python bench.py --scene $scene --width $w --height $h --spp $spp \
      --depth $depth --steps $steps --warmup 1 --no-cpu-baseline > $log 2>&1 || { echo "$scene n$n rc=$?"; tail -20 $log; exit 1; }
    echo "{\"emu\": $n, \"scene\": \"$scene\", \"line\": $(grep '^{' $log | tail -1)}" >> $OUT
    grep '^{' $log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$scene', 'n=$n', 'step', d['ms_per_step'], 'Mrays/s', d['value'])"
  done
done
