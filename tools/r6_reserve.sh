# usage: bash tools/r6_reserve.sh <tag>: the multi-rank GPU tests, then the exchange rehearsal of one
# rank's share (--shard-of N --force-exchange) at the default thresholds
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "${K:-dist_gloo or pipelined_ranks or collapse}" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
MIDS=65536 SHARDS="1 2 4 8" EXTRA="--force-exchange" bash tools/r6_midsweep.sh $1/fx || exit 1
MIDS=65536 SHARDS="2 4 8" bash tools/r6_midsweep.sh $1/plain
