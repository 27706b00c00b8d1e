# GPU iteration: a pytest selection, the driver's bench command, the merge phase timeline
# usage: bash tools/r2_step.sh <tag> "<pytest args>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $2 > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 && echo BENCH_OK && grep '^{' $OUT/bench_driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'kern',d['kernels'])" || exit 1
timeout -k 10 300 python3 tools/debug/merge_timeline.py 100000 1,6,20,200,800 > $OUT/timeline.log 2>&1 && echo TIMELINE_OK
