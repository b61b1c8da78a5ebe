set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --sync-check-steps 0 > gpurun_out/ch_A$r.json 2> gpurun_out/ch_A$r.log || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --sync-check-steps 0 --chunk-paths 268435456 > gpurun_out/ch_B$r.json 2> gpurun_out/ch_B$r.log || exit 1
done
