# round 4: the quirk scenes of the oracle's known-answer tests through both kernels
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "quirk_scenes or equal_t_within" > $O/tests.log 2>&1
