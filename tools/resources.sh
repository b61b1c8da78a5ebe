#!/bin/bash
# Per-kernel VGPR / scratch / occupancy of render.hip as compiled for gfx950 (extra defines as args).
cd "$(dirname "$0")/../ba_pathtracing_fur_amd/csrc"
/opt/rocm/bin/hipcc -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize "$@" -c render.hip \
  -o /tmp/khp_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*(Function Name|VGPRs|ScratchSize \[bytes\/lane\]|Occupancy \[waves\/SIMD\]): ([^ ]+).*/\2/' |
  paste - - - - | awk '{printf "%-60s vgpr %4s scratch %4s waves %s\n", $1, $2, $3, $4}' | grep -E "${KHP_RES_FILTER:-extend|shadow|shade|k_shade}"
