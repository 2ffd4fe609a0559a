set -e
timeout -k 10 300 python3 tools/ab_bench.py --scene sphere:6 --spp 8 --reps 2 --no-parity s1:opt2=1 s2:opt2=2 s4:opt2=4 s8:opt2=8 | tail -n 1
timeout -k 10 300 python3 tools/ab_bench.py --scene random:1000000 --spp 8 --reps 2 --no-parity s1:opt2=1 s2:opt2=2 s4:opt2=4 s8:opt2=8 | tail -n 1
