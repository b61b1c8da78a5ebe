# round 4 (l): rank-of-8 frame time vs the two-level records' first bounce (wide_from) and the longest-first threshold
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04l
mkdir -p $O
cd $R
for v in "wide_from=2" "wide_from=1" "wide_from=0" "wide_from=2 heavy_iters=80" "wide_from=2 heavy_iters=320" "wide_from=2"; do
  tag=$(echo $v | tr ' =' '_-')
  timeout -k 10 200 python -u tools/scale_probe.py --nranks 8 --steps 20 --set $v > $O/scale_$tag.json 2> $O/scale_$tag.err
done
