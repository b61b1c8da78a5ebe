# round 4 (v): synchronous calls (1-spp GUI, 8-spp pass) through the wavefront with the two-level records from bounce 0/1/2
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v
mkdir -p $O
cd $R
for cfg in "0 2" "1 2" "1 1" "1 0" "0 0"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 150 python3 tools/sync_trace.py 6 $cfg > $O/st_$tag.json 2> $O/st_$tag.log
done
