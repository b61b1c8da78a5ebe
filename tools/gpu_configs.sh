set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multigpu.py -x -v --timeout 400 --timeout-method thread -k "config1_full or config2_full or config5_full or multigpu or bench_launches or rccl" > gpurun_out/cfg_tests_r02d.log 2>&1 && \
for c in 1 2 3 5; do timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_cfg${c}_r02d.json 2> gpurun_out/bench_cfg${c}_r02d.log || exit 1; done
