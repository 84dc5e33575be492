# Round-4 GPU check on the tree as committed: the -m gpu suite, smoke, bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04g bash scripts/gpu_check.sh
