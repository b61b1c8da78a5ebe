# round 4: the driver's 20 passes as ONE chunk (chunk_paths 2^29, 332M paths) vs the automatic 2 chunks
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04af
mkdir -p $O
cd $R
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > $O/auto_$r.json 2> $O/auto_$r.log
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 --chunk-paths 536870912 > $O/one_$r.json 2> $O/one_$r.log
done
