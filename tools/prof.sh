# usage: bash tools/prof.sh <tag> [bench args...]
# rocprofv3 kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-replay "$@" > $OUT/bench_trace.log 2>&1 && echo TRACE_OK && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --no-replay --no-profile "$@" > $OUT/bench_fetch.log 2>&1 && echo FETCH_OK && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu-baseline --no-replay --no-profile "$@" > $OUT/bench_write.log 2>&1 && echo WRITE_OK
