#!/bin/bash
# A/B library builds ab/<name>.so on the device-memory scenes, alternating processes:
#   LIBS="base new" AB_SCENES="sphere:6 random:10000000" AB_ITERS=2 tools/ab_libs_scenes.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for S in ${AB_SCENES:-sphere:6 random:10000000}; do
  n=${S//:/_}
  for i in $(seq 1 ${AB_ITERS:-2}); do
    for L in ${LIBS:-base new}; do
      PTAMD_LIB=ab/$L.so timeout -k 10 ${AB_TIMEOUT:-200} python3 tools/ab_bench.py --scene $S --reps ${AB_REPS:-3} ${AB_ARGS:-v:} > gpurun_out/abl_${n}_$L.$i.log 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/abl_${n}_$L.$i.log; exit 1; }
      echo "$S $L $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abl_${n}_$L.$i.log') if l.startswith('{')][-1]); print({k: round(v['mean_ms'],2) for k,v in d['results'].items()}, d.get('frame_sha1'))")"
    done
  done
done
