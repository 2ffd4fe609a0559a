#!/bin/bash
# The scene legs' own timed frames (bench.py --leg, the leg's contexts and
# grid) under library builds ab/<name>.so, alternating: config 3 and 5 at
# BASELINE's camera.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for leg in ${LEGS:-config3 config5}; do
  for i in 1 2; do
    for L in ${LIBS:-base new}; do
      PTAMD_LIB=ab/$L.so timeout -k 10 200 python3 bench.py --leg $leg --leg-camera ref --steps ${STEPS:-12} \
        > gpurun_out/legab_${leg}_$L.$i.log 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/legab_${leg}_$L.$i.log; exit 1; }
      echo "$leg $L $(tail -1 gpurun_out/legab_${leg}_$L.$i.log | cut -c1-200)"
    done
  done
done
