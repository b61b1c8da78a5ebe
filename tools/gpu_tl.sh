set -o pipefail
# timeline of one rank-of-N frame (rank 0 of NR tiles) under rocprofv3 --kernel-trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/tl
cd /tmp && export TMPDIR=/tmp
for nr in ${NRS:-8 1}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl/n$nr -o run -- python3 $R/tools/scale_probe.py --nranks $nr --ranks-max 1 --steps 2 > $R/gpurun_out/tl/n$nr.json 2>&1 || exit 1
  python3 $R/tools/timeline.py $(ls $R/gpurun_out/tl/n$nr/*kernel_trace.csv $R/gpurun_out/tl/n$nr/*/*kernel_trace.csv 2>/dev/null | head -1) 1 > $R/gpurun_out/tl/n$nr.txt || exit 1
  tail -1 $R/gpurun_out/tl/n$nr.txt
done
