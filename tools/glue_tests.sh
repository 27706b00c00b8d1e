# usage: bash tools/glue_tests.sh <tag>: the glue-optimisation GPU tests with their printed drift
# statistics (-s), outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests/test_glue.py -m gpu -v -s --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
exit $rc
