# round 4: rocprof passes of the driver's batch shape (20 fused passes per timed batch: 2 chunks of 10 frames)
set -e
R=$GRAFT_REPO_ROOT
cd $R
STEPS=20 bash tools/profile.sh r04dc trace fetch write
