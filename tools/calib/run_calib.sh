#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (GPU box, via gpurun, from the repo root)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib
mkdir -p $OUT
make -s -C $R/tools/calib
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/calib/calib_gather > $OUT/plain.json
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $R/tools/calib/calib_gather > $OUT/fetch.json 2> $OUT/fetch.log
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $R/tools/calib/calib_gather > $OUT/write.json 2> $OUT/write.log
echo calib done
