# round 4 (final): the driver's command three times (run-to-run spread), and configs 3 and 5 at HEAD
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04final
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_$i.json 2> $O/driver_$i.log
done
timeout -k 10 300 python3 bench.py --config 3 --no-cpu-baseline > $O/cfg3.json 2> $O/cfg3.log
timeout -k 10 400 python3 bench.py --config 5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.log
