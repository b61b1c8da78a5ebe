#!/bin/bash
# Build libkirk_hip.so with extra compile definitions into ba_pathtracing_fur_amd/lib/variants/<name>/
# for A/B runs (KHP_LIB=<that .so> python bench.py ...).  usage: tools/build_variant.sh <name> -DFOO=1 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
C=$R/ba_pathtracing_fur_amd/csrc
O=$R/ba_pathtracing_fur_amd/lib/variants/$NAME
mkdir -p $O
FL="-O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wall -Wno-unused-function --offload-arch=gfx950 -fno-slp-vectorize"
/opt/rocm/bin/hipcc $FL "$@" -c ${SRC:-$C/render.hip} -o $O/render.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $O/libkirk_hip.so $O/render.o $R/ba_pathtracing_fur_amd/lib/obj/scene.o \
  $R/ba_pathtracing_fur_amd/lib/obj/bvh_build.o $R/ba_pathtracing_fur_amd/lib/obj/flatten.o -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
echo "built $O/libkirk_hip.so ($*)"
