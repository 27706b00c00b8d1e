# usage: bash tools/prof_window.sh <tag> [bench args...]
# rocprofv3 kernel trace + stats of the bench command, then one PMC pass each for
# FETCH_SIZE and WRITE_SIZE (they cannot share a pass); tools/prof_window.py then
# keeps only the dispatches between bench.py's two k_window_mark launches (the timed region)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
echo "$*" > $OUT/bench_args.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-replay "$@" > $OUT/bench_trace.log 2>&1 && echo TRACE_OK && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --no-replay --no-profile "$@" > $OUT/bench_fetch.log 2>&1 && echo FETCH_OK && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline --no-replay --no-profile "$@" > $OUT/bench_write.log 2>&1 && echo WRITE_OK && \
python3 tools/prof_window.py $OUT > $OUT/window.json && echo SUMMARY_OK
