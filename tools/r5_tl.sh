# usage: bash tools/r5_tl.sh <tag> <lib.so>: phase timelines of the heavy merges (merge_timeline.py)
# and of the middle regime (mid_fused_timeline.py) with that library; outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
GEOBPE_LIB=$PWD/$2 timeout -k 10 200 python3 tools/debug/merge_timeline.py 100000 6,20 > $OUT/timeline_$(basename $2).txt 2>&1 && \
GEOBPE_LIB=$PWD/$2 timeout -k 10 200 python3 tools/debug/mid_fused_timeline.py 100,400 > $OUT/mid_timeline_$(basename $2).txt 2>&1
