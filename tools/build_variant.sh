#!/bin/bash
# usage: tools/build_variant.sh NAME [extra hipcc flags for render.hip]
# -> ba_pathtracing_fur_amd/lib/libkirk_hip_NAME.so (A/B with tools/gpu_ab2.sh NAME; KHP_LIB selects it)
set -e
cd "$(dirname "$0")/../ba_pathtracing_fur_amd/csrc"
n=$1; shift
O=../lib/obj
make -s ../lib/libkirk_hip.so >/dev/null
/opt/rocm/bin/hipcc -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wall -Wno-unused-function \
  --offload-arch=gfx950 -fno-slp-vectorize "$@" -c render.hip -o /tmp/khp_render_$n.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lib/libkirk_hip_$n.so $O/scene.o /tmp/khp_render_$n.o \
  $O/bvh_build.o $O/flatten.o -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
echo ../lib/libkirk_hip_$n.so
