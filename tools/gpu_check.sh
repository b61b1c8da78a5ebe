set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02w.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02w.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r02w.json 2> gpurun_out/bench_r02w.log || exit 1
