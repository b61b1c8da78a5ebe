# round 4 (m): rank-of-8 and 1-GPU frame time with two fused batches in flight, half grids (library) or full grids (probe build)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m
mkdir -p $O
cd $R
run() {  # tag, env..., -- args
  tag=$1; shift
  timeout -k 10 240 env "$@" > $O/$tag.json 2> $O/$tag.err
}
run base_s20 python -u tools/scale_probe.py --nranks 1 8 --steps 20
run f2h_s20 GPU_MAX_HW_QUEUES=8 python -u tools/scale_probe.py --nranks 1 8 --steps 20 --set frames_in_flight=2 fuse_frames=10
run f2f_s20 GPU_MAX_HW_QUEUES=8 KHP_LIB=$R/variants/libkirk_fullgrid.so python -u tools/scale_probe.py --nranks 1 8 --steps 20 --set frames_in_flight=2 fuse_frames=10
run base_s40 python -u tools/scale_probe.py --nranks 1 8 --steps 40 --set fuse_frames=20
run f2f_s40 GPU_MAX_HW_QUEUES=8 KHP_LIB=$R/variants/libkirk_fullgrid.so python -u tools/scale_probe.py --nranks 1 8 --steps 40 --set frames_in_flight=2 fuse_frames=20
run base_s20b python -u tools/scale_probe.py --nranks 1 8 --steps 20
