#!/bin/bash
# Build a variant of libkirk_hip.so with extra -D flags for an A/B on the GPU box
# (bench.py / tests pick it up with KHP_LIB=<path>).  Run here, on the CPU, after
# the regular build (it links the regular scene/bvh/flatten objects).
# usage: [SRC=/abs/path/render.hip] tools/build_variant.sh <name> -DKHP_EXT_REFILL=32 ...   -> variants/libkirk_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/variants"
cd "$R/ba_pathtracing_fur_amd/csrc"
/opt/rocm/bin/hipcc -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wall -Wno-unused-function \
  --offload-arch=gfx950 -fno-slp-vectorize -I. "$@" -c "${SRC:-render.hip}" -o "$R/variants/render_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$R/variants/libkirk_$NAME.so" "$R/variants/render_$NAME.o" \
  ../lib/obj/scene.o ../lib/obj/tonemap_host.o ../lib/obj/bvh_build.o ../lib/obj/flatten.o -L/opt/rocm/lib -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
rm -f "$R/variants/render_$NAME.o"
echo "$R/variants/libkirk_$NAME.so"
