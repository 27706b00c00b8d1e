set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh && bash tools/prof.sh "$1"
