set -e
LIBS="prev new" AB_ARGS="--no-parity cull:lds=1,opt3=1" bash tools/ab_libs.sh
