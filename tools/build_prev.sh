#!/bin/bash
# Build libptamd.so of a git revision into ab/<name>.so for A/B timing:
#   tools/build_prev.sh NAME [REV=HEAD]
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=${2:-HEAD}
rm -rf ab/tree_$name && mkdir -p ab/tree_$name
git archive "$rev" | tar -x -C ab/tree_$name
make -s -C ab/tree_$name/discovering-path-tracer_amd libptamd.so
cp ab/tree_$name/discovering-path-tracer_amd/libptamd.so ab/$name.so
rm -rf ab/tree_$name
echo "built ab/$name.so from $rev"
