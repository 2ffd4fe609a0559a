#!/bin/bash
# 1-GPU box: the root's step of an N-GPU gather run, emulated
# (PT_BENCH_EMULATE_RANKS: its tile share, render+pack, unpack of N slots, no
# transfer) under bench variants; then the real exchange path at N=1 over
# RCCL and the gloo rehearsal of N=2/4 (--verify).
# VARIANTS: space-separated "name:bench args with commas for spaces".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/emu_${TAG:-x}.jsonl
: > $OUT
STEPS=${STEPS:-50}
VARIANTS=${VARIANTS:-"base:"}
for n in ${RANKS:-1 2 4 8}; do
  for v in $VARIANTS; do
    name=${v%%:*}; args=${v#*:}; args=${args//,/ }
    log=gpurun_out/emu_n${n}_$name.log
    PT_BENCH_EMULATE_RANKS=$n timeout -k 10 120 python bench.py --steps $STEPS --warmup 3 --no-cpu-baseline $args \
      > $log 2>&1 || { echo "emu n$n $name rc=$?"; tail -20 $log; exit 1; }
    echo "{\"emu\": $n, \"variant\": \"$name\", \"line\": $(grep '^{' $log | tail -1)}" >> $OUT
    grep '^{' $log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('n=$n', '$name', 'step', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'host', d['host_issue_ms_per_step'])"
  done
done
if [ "${SKIP_DIST:-0}" = "1" ]; then exit 0; fi
MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 PT_BENCH_FORCE_DIST=1 timeout -k 10 120 python bench.py --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/force_dist.log 2>&1 \
  || { echo "force dist rc=$?"; tail -20 gpurun_out/force_dist.log; exit 1; }
grep '^{' gpurun_out/force_dist.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('force_dist', d['ms_per_step'], d['roofline']['kernel_ms'], d['host_issue_ms_per_step'])"
for n in 2 4; do
  PT_BENCH_DEVICE=0 PT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 --verify \
    > gpurun_out/rehearsal_n${n}.log 2>&1 || { echo "n$n rc=$?"; tail -30 gpurun_out/rehearsal_n${n}.log; exit 1; }
  grep '^{' gpurun_out/rehearsal_n${n}.log | tail -1 | grep -o "verified[^,]*"
done
