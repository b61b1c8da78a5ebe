set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --config 5 --steps 4 --warmup 1 --sync-check-steps 1 --no-cpu-baseline"
$B --fuse 1 > gpurun_out/c5_fuse1.json 2> gpurun_out/c5_fuse1.log && \
$B --fuse 4 --chunk-paths 33554432 > gpurun_out/c5_fuse4_c25.json 2> gpurun_out/c5_fuse4_c25.log && \
$B --fuse 2 > gpurun_out/c5_fuse2.json 2> gpurun_out/c5_fuse2.log && \
timeout -k 10 300 python -u bench.py --config 3 --spp 32 --steps 4 --warmup 1 --sync-check-steps 1 --no-cpu-baseline > gpurun_out/c3_spp32.json 2> gpurun_out/c3_spp32.log
