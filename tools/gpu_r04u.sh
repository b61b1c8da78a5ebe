# round 4 (u): a synchronous 8-spp pass split into batches in flight (half / full grids) vs one call
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04u
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=8
timeout -k 10 200 python -u tools/split_sync_probe.py 6 2 > $O/half2.json 2> $O/half2.err
KHP_LIB=$R/variants/libkirk_fullgrid.so timeout -k 10 200 python -u tools/split_sync_probe.py 6 2 > $O/full2.json 2> $O/full2.err
