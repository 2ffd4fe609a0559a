set -e
LIBS="prev new" AB_ARGS="--no-parity cull:lds=1 s4:lds=1,opt2=4 d0:lds=1,depth=0" bash tools/ab_libs.sh
