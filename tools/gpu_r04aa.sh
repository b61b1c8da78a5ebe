# round 4: synchronous calls of 1-8 spp, wavefront vs path kernel (threshold of the automatic choice)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04aa
mkdir -p $O
cd $R
for r in 1 2; do
  timeout -k 10 240 python3 tools/sync_spp_probe.py > $O/spp_$r.json 2> $O/spp_$r.log
done
