# Round-4 final check on the tree as committed: the -m gpu suite, smoke, bench, then the bench under a
# kernel trace with the fingerprint kernel's FETCH/WRITE passes (scripts/profile_round.sh).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04n bash scripts/gpu_check.sh || exit $?
R=r04n bash scripts/profile_round.sh
