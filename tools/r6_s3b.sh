# usage: bash tools/r6_s3b.sh <tag> <libs...>: tools/r5_step.sh over the libraries (parity subset on the last,
# A/B, trace), then tools/r6_s3.sh (the whole GPU suite, smoke, bench lines, the two-replica window) with
# the tree's own library
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
bash tools/r5_step.sh ${TAG}_ab "$@" && bash tools/r6_s3.sh ${TAG}_suite
