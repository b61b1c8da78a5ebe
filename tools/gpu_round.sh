set -o pipefail
# usage (on the GPU box): TAG=r02e bash tools/gpu_round.sh  -> GPU tests, metric bench line, config-5 bench line
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log && \
timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/bench_cfg5_$TAG.json 2> gpurun_out/bench_cfg5_$TAG.log
