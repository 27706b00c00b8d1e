# usage: bash tools/fx.sh <tag> [pytest -k expr]: the multi-rank tests (engine-owned exchange over
# gloo on one GPU), then the 1-GPU RCCL rehearsal of the N > 1 loop (--force-exchange) on the driver
# window and the default run, and a kernel trace of the default forced-exchange run; outputs under
# gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
K=${2:-"dist_gloo or pipelined_ranks or test_bench"}
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$K" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEF_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --force-exchange > $OUT/bench_fx_window.json 2> $OUT/bench_fx_window.err && echo FXW_OK && \
timeout -k 10 300 python3 bench.py --gpus 1 --force-exchange > $OUT/bench_fx_default.json 2> $OUT/bench_fx_default.err && echo FXD_OK && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p -o run -- python3 bench.py --gpus 1 --force-exchange > $OUT/bench_prof.json 2> $OUT/bench_prof.err && echo PROF_OK
