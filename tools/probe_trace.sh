#!/bin/bash
# rocprofv3 kernel trace of a short fused bench run, for a library variant (run on the GPU box)
# usage: tools/probe_trace.sh <tag> [library]   -> gpurun_out/ptrace_<tag>/
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LIB=${2:+$R/$2}
mkdir -p $R/gpurun_out/ptrace_$TAG
cd /tmp && export TMPDIR=/tmp
KHP_LIB=$LIB timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ptrace_$TAG -o run -- python3 $R/bench.py --no-cpu-baseline --sync-check-steps 0 --iso-steps 0 --gui-steps 0 --steps 8 --warmup 8 > $R/gpurun_out/ptrace_$TAG/bench.json 2> $R/gpurun_out/ptrace_$TAG/bench.log
