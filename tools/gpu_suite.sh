# usage: bash tools/gpu_suite.sh <tag>: the whole GPU suite, smoke, the driver bench window with
# sampled events and without events, the default bench; outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 && echo SMOKE_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err && echo BENCH_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-profile --no-replay --no-cpu-baseline > $OUT/bench_noprof.json 2> $OUT/bench_noprof.err && echo NOPROF_OK && \
timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEFAULT_OK
