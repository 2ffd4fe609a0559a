set -e
LIBS="prev new" AB_ARGS="--no-parity --scene sphere:5 --spp 2 s:lds=0" bash tools/ab_libs.sh
