set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04ae
cd $R
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $R/gpurun_out/r04ae/bench_driver_cmd.json 2> $R/gpurun_out/r04ae/bench_driver_cmd.log
