# usage: bash tools/r3_iter.sh <tag> <pytest -k expr>: GPU tests, the default bench, the middle-regime
# phase timeline; outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3_$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu ${XFLAG--x} -v --timeout 600 --timeout-method thread -k "$2" > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEF_OK && \
timeout -k 10 200 python3 tools/debug/mid_timeline.py 150,400,800 16384 > $OUT/timeline.txt 2>&1 && echo TL_OK
