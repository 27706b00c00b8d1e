# usage: bash tools/r3_check.sh <tag> [pytest -k expr]
# bench launcher + world-8 pipelined tests, then the driver's bench command with and without
# per-launch HIP events (event overhead), outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
K=${2:-"test_bench or pipelined_ranks"}
OUT=gpurun_out/r3_$TAG
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "$K" > $OUT/pytest.txt 2>&1 && echo TESTS_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err && echo BENCH_OK && \
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-profile --no-replay --no-cpu-baseline > $OUT/bench_noprof.json 2> $OUT/bench_noprof.err && echo NOPROF_OK && \
timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEFAULT_OK
tail -3 $OUT/pytest.txt
