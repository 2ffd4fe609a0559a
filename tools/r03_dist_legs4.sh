#!/bin/bash
# 1-GPU box: bench.py's N>1 path with 4 ranks on device 0 over gloo (the box
# frame's sparse gather with --verify, then configs 4 and 5 split across the
# ranks and reduced, each checked bitwise on rank 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dist_legs4_${TAG:-x}
mkdir -p $OUT
PT_BENCH_DEVICE=0 PT_BENCH_BACKEND=gloo timeout -k 10 ${LEG_TIMEOUT:-700} python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 4 --steps 20 --warmup 3 --verify \
  > $OUT/bench_n4.log 2>&1 || { echo "n4 rc=$?"; tail -30 $OUT/bench_n4.log; exit 1; }
grep '^{' $OUT/bench_n4.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('box', d['ms_per_step'], d.get('verified_bitwise_vs_single_gpu'), d.get('bench_wall_s'))
for k,c in d.get('configs',{}).items(): print(k, {x: c.get(x) for x in ('ms_per_step','verified_bitwise_vs_single_gpu','setup_s','counting_passes_s','error')})
"
