set -e
run() { tag=$1; shift; timeout -k 10 600 python3 bench.py "$@" --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo "$tag rc=$?"; tail -20 gpurun_out/bench_$tag.log; exit 1; }; echo "$tag $(grep '^{' gpurun_out/bench_$tag.log | tail -1)"; }
run sphere --scene sphere --steps 3 --warmup 1
run sphere4k --scene sphere --width 3840 --height 2160 --spp 16 --depth 8 --steps 1 --warmup 1
run syn1m --scene synthetic:1000000 --steps 2 --warmup 1
run syn10m --scene synthetic:10000000 --spp 1 --steps 1 --warmup 1
