#!/bin/bash
# round 6: the emulated root step with RCCL's own grouped self send/recv per
# frame (PT_DIST_EMU_P2P=1) against the device-copy stand-in: RCCL's host and
# device cost per frame at N = 2/4/8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06q}; mkdir -p $OUT
for n in 8 4 2; do
  for v in 0 1; do
    PT_DIST_EMU_P2P=$v PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-scene-legs > $OUT/emu${n}_p2p$v.log 2>&1 || { echo "emu$n p2p$v rc=$?"; tail $OUT/emu${n}_p2p$v.log; exit 1; }
    grep "bench detail" $OUT/emu${n}_p2p$v.log | sed 's/^bench detail: //' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('N=$n p2p=$v', d['ms_per_step'], 'host', d['host_issue_ms_per_step'])"
  done
done
