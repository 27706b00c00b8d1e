# usage: bash tools/r5_step2.sh <tag> <lib.so>...: tools/r5_step.sh, then the held-out glue fixture's
# device test and the heavy-merge / middle-regime timelines of the last library
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
LAST=${@: -1}
bash tools/r5_step.sh $TAG "$@" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_glue.py -m gpu -x -v --timeout 500 --timeout-method thread -k heldout > gpurun_out/$TAG/pytest_heldout.txt 2>&1; echo "heldout rc=$?"
bash tools/r5_tl.sh $TAG $LAST
