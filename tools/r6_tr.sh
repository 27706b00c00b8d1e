# usage: bash tools/r6_tr.sh <tag> <bench args...>: a kernel trace of one bench run (outputs under gpurun_out/<tag>/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile "$@" > $OUT/b.json 2> $OUT/b.err && echo TR_OK
python3 tools/trace_window.py $OUT/tr > $OUT/window.txt; head -20 $OUT/window.txt
