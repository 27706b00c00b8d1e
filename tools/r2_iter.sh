# iteration GPU check: selected GPU tests, the driver's bench command, an apply/mark
# phase timeline of the driver's window, optionally a kernel trace
# usage: bash tools/r2_iter.sh <tag> "<pytest args>" [trace]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread $2 > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 && echo BENCH_OK && grep '^{' $OUT/bench_driver.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'ms',d['ms_per_step'],'kern',d['kernels'],'roof',d['roofline']['frac'] if d['roofline'] else None)" || exit 1
timeout -k 10 300 python3 tools/debug/apply_timeline.py 100000 6,12,20 > $OUT/timeline.log 2>&1 && echo TIMELINE_OK || exit 1
if [ "$3" = "trace" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-replay > $OUT/bench_trace.log 2>&1 && echo TRACE_OK
fi
