set -o pipefail
# usage (on the GPU box): TAG=r01h bash tools/gpu_round.sh  -> GPU tests, bench line, rocprof trace + FETCH_SIZE passes
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log && \
bash tools/profile.sh $TAG ${PASSES:-trace fetch}
