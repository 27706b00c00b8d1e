# usage: bash tools/r6_ab3.sh <tag> <libs...>: tools/r5_step.sh over the libraries, then the multi-rank tests
# with the tree's own library
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
PYTEST_K="c3_1000 or test_gpu_parity" bash tools/r5_step.sh $TAG "$@" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "dist_gloo or pipelined_ranks or collapse" > gpurun_out/$TAG/pytest_multi.txt 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_multi.txt
exit $rc
