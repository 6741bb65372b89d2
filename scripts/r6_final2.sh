cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu.sh r6w graph c5graph || exit 1
bash scripts/r6_final_tests.sh
