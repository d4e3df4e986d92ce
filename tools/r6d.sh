# round 5: DP2 rehearsal kernel timeline, then the whole GPU test suite (with durations)
bash tools/r6c.sh || exit $?
cd $GRAFT_REPO_ROOT
TAG=r6d bash tools/gpu.sh tests
