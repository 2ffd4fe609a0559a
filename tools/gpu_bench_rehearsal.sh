#!/bin/bash
# 1-GPU box: the N=1 bench, then the N=2/N=4 code paths rehearsed with gloo and
# every rank on device 0 (RCCL needs one GPU per rank; the driver runs the
# real N>1 benches on an 8-GPU node).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_n1.log 2>&1 || { echo "n1 rc=$?"; tail -20 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
for n in 2 4; do
  for coll in gather reduce; do
    PT_BENCH_DEVICE=0 PT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 --verify --collective $coll \
      > gpurun_out/bench_n${n}_$coll.log 2>&1 || { echo "n$n $coll rc=$?"; tail -30 gpurun_out/bench_n${n}_$coll.log; exit 1; }
    grep '^{' gpurun_out/bench_n${n}_$coll.log | tail -1 | grep -o "verified[^,]*"
  done
done
