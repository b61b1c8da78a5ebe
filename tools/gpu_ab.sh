set -o pipefail
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/gpu_tests.log
bash tools/ab.sh ${AB:-base}
