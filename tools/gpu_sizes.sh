set -o pipefail
# k_extend records/s against tree size (config-3 scene with N strands), metric resolution
TAG=${TAG:-r03}
mkdir -p gpurun_out
for n in ${SIZES:-30 300 3000 30000 300000 1000000}; do
  timeout -k 10 300 python -u bench.py --strands $n --steps 16 --warmup 8 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 > gpurun_out/size_${n}_$TAG.json 2> gpurun_out/size_${n}_$TAG.log || exit 1
  echo "size $n done"
done
