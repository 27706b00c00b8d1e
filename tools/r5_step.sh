# usage: bash tools/r5_step.sh <tag> <lib.so>...: the GPU parity subset (tests/test_gpu_parity.py,
# tests/test_tail.py) with the LAST library, the A/B of all of them (tools/ab.sh: driver window
# twice + default run once each), then a kernel trace of the driver window with the last one;
# outputs under gpurun_out/<tag>/ and gpurun_out/ab_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
LAST=${@: -1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
GEOBPE_LIB=$PWD/$LAST timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tail.py -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/ab.sh $TAG "$@" || exit 1
GEOBPE_LIB=$PWD/$LAST timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-replay --steps 20 --warmup 5 > $OUT/bench_trace.log 2>&1 && echo TRACE_OK
