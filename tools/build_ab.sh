#!/bin/bash
# Build an A/B variant of libptamd.so with extra device defines:
#   tools/build_ab.sh NAME [-DFOO ...]   ->  ab/NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab/obj_$name
make -s -C discovering-path-tracer_amd build/pt_api.o build/pt_group.o build/scene/bvh.o build/scene/light.o build/scene/camera.o build/scene/obj_loader.o build/scene/wide_bvh.o
D=discovering-path-tracer_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero ${DEVFLAGS--fno-slp-vectorize} -I include -I $D/csrc "$@" \
  -c ${SRC:-$D/csrc/pt_device.hip} -o ab/obj_$name/pt_device.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$name.so ab/obj_$name/pt_device.o \
  $D/build/pt_api.o $D/build/pt_group.o $D/build/scene/bvh.o $D/build/scene/light.o $D/build/scene/camera.o $D/build/scene/obj_loader.o $D/build/scene/wide_bvh.o -lpthread
echo "built ab/$name.so"
