# usage: bash tools/r3_run.sh <tag> <pytest -k expr | -> [bench args...]
# GPU tests selected by -k (skipped with "-"), then bench.py with the given arguments;
# outputs under gpurun_out/r3_<tag>/ (a heartbeat file keeps quiet phases alive)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
K=$2
shift 2
OUT=gpurun_out/r3_$TAG
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ "$K" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$K" > $OUT/pytest.txt 2>&1
  rc=$?
  tail -4 $OUT/pytest.txt
  [ $rc -eq 0 ] || exit $rc
  echo TESTS_OK
fi
if [ $# -gt 0 ]; then
  timeout -k 10 300 python3 bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err && echo BENCH_OK && cat $OUT/bench.json | head -c 1500
fi
