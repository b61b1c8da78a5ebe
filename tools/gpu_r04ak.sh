# round 4: k_shadow_finish on its own occupancy grid (variant finown) vs k_shade's (512-thread) grid
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ak
mkdir -p $O
cd $R
for r in 1 2 3; do
  for v in base finown; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 300 env ${L:+KHP_LIB=$L} python3 bench.py --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.log
    timeout -k 10 300 env ${L:+KHP_LIB=$L} python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > $O/d_${v}_$r.json 2> $O/d_${v}_$r.log
  done
done
