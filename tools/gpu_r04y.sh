# round 4 (y): k_shade / k_shadow_finish / k_accumulate_all measured HBM traffic (FETCH_SIZE, WRITE_SIZE passes) + kernel trace
set -e
R=$GRAFT_REPO_ROOT
cd $R
KREGEX="k_shade|k_shadow_finish|k_accumulate" bash tools/profile.sh r04y trace fetch write
