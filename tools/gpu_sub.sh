set -o pipefail
# sub-frame A/B on the GPU box: parity tests for path sets, bench at KHP_SUBFRAMES=1..4, scale probe
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "subframes or chunking or shards or frame_parity" > gpurun_out/gpu_sub_tests.log 2>&1 || { tail -30 gpurun_out/gpu_sub_tests.log; exit 1; }
tail -2 gpurun_out/gpu_sub_tests.log
for k in ${KS:-1 2 3 4}; do
  KHP_SUBFRAMES=$k timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline 2>/dev/null > gpurun_out/sub_$k.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sub_$k.json')); f=d['frame']; print('K=$k', d['value'], 'ms', d['ms_per_step'], 'ext', f['extend_ms'], 'sh', f['shadow_ms'], 'frac', d['roofline']['frac'], 'avg', d['roofline']['avg_launch_ms'])"
done
for k in ${PK:-2}; do
  KHP_SUBFRAMES=$k timeout -k 10 300 python3 tools/scale_probe.py --steps 3 > gpurun_out/scale_probe_k$k.json 2>/dev/null || exit 1
  echo "probe K=$k"; grep nranks gpurun_out/scale_probe_k$k.json | grep -v scale_probe
done
