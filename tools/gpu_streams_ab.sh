#!/bin/bash
# 1-GPU box: A/B of 1..4 alternating streams on the gather path (emulated
# root step of N ranks, PT_BENCH_EMULATE_RANKS) and at N=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/streams_${TAG:-x}.jsonl
: > $OUT
STEPS=${STEPS:-100}
run() {   # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 python bench.py --steps $STEPS --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_$name.log 2>&1 \
    || { echo "$name rc=$?"; tail -20 gpurun_out/ab_$name.log; exit 1; }
  echo "{\"name\": \"$name\", \"line\": $(grep '^{' gpurun_out/ab_$name.log | tail -1)}" >> $OUT
  grep '^{' gpurun_out/ab_$name.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', 'step', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'host', d['host_issue_ms_per_step'])"
}
for n in ${RANKS:-1 2 4 8}; do
  for v in ${VARIANTS:-s1:--streams,1 s2:--streams,2}; do
    name=${v%%:*}; args=${v#*:}; args=${args//,/ }
    if [ $n = 1 ]; then run n1_$name X=1 $args; else run emu${n}_$name PT_BENCH_EMULATE_RANKS=$n $args; fi
  done
done
