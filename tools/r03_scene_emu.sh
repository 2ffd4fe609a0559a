#!/bin/bash
# 1-GPU box: rank 0's step of an N-GPU tile split (PT_BENCH_EMULATE_RANKS,
# equal shares) for the large-scene configs, frame time only (--profile-run:
# no counting passes), with option variants.  Output: one line per run.
#   SPECS="sphere 1920 1080 8 4 3;..." RANKS="1 8" VARIANTS="base 13=2" tools/r03_scene_emu.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/scene_emu_${TAG:-x}
mkdir -p $OUT
IFS=';' read -ra specs <<< "${SPECS:-sphere 1920 1080 8 4 3;sphere 3840 2160 16 8 2;synthetic:10000000 1920 1080 8 4 3}"
for spec in "${specs[@]}"; do
  read -r scene w h spp depth steps <<< "$spec"
  for n in ${RANKS:-1 8}; do
    for v in ${VARIANTS:-base}; do
      opt=""; [ "$v" != "base" ] && for kv in ${v//,/ }; do opt="$opt --opt $kv"; done
      log=$OUT/$(echo $scene | tr ':' '_')_${w}_${spp}_n${n}_${v//[=,]/_}.log
      PT_BENCH_EMULATE_RANKS=$n timeout -k 10 300 python bench.py --scene $scene --width $w --height $h --spp $spp \
        --depth $depth --steps $steps --warmup 1 --no-cpu-baseline --profile-run $opt > $log 2>&1 \
        || { echo "$scene n$n $v rc=$?"; tail -20 $log; exit 1; }
      grep '^{' $log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$scene ${w}x$h ${spp}spp D$depth', 'n=$n', '$v', 'ms', d['ms_per_step'])"
    done
  done
done
