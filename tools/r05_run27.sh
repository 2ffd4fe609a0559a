#!/bin/bash
# round-5 GPU call 27: the sample-lane auto rule changed for split frames
# (LDS scenes: 2 lanes on 2-7 ranks, 4 on 8+): parity and multi-rank GPU
# tests, then the emulated box root step at N = 2/4/8 with the defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05zd; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_group.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for n in 2 4 8; do
  PT_BENCH_EMULATE_RANKS=$n timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-scene-legs --no-cpu-baseline > $OUT/emu$n.log 2>&1 || { echo "emu $n rc=$?"; tail -5 $OUT/emu$n.log; exit 1; }
  grep '^{' $OUT/emu$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d.get('host_issue_ms_per_step'), d.get('verified_vs_oracle'))" | tee -a $OUT/emu_box.log
done
