# usage: bash tools/r5_base.sh <tag>: the driver window bench, the default bench, the heavy-merge
# phase timeline and a kernel trace of the window; outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err && echo BENCH_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --no-cpu-baseline --no-replay > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEFAULT_OK && \
timeout -k 10 240 python3 tools/debug/merge_timeline.py 100000 6,10,20 > $OUT/timeline.txt 2>&1 && echo TL_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-replay --steps 20 --warmup 5 > $OUT/bench_trace.log 2>&1 && echo TRACE_OK
