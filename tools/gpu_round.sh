set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r01g.json 2> gpurun_out/bench_r01g.log && \
bash tools/profile.sh r01g trace fetch
