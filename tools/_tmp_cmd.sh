PT_BENCH_DEVICE=0 PT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 2 --warmup 1 --verify --collective reduce > gpurun_out/bench_n2_reduce.log 2>&1
grep -a "verify\|verified" gpurun_out/bench_n2_reduce.log | head -3
