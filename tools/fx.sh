# usage: bash tools/fx.sh <tag> [pytest -k expr]: the multi-rank tests (engine-owned exchange over
# gloo on one GPU), then the 1-GPU rehearsal of the N > 1 loop (--force-exchange: the whole protocol
# at world size 1) on the driver window and the default run, with the peer exchange (default) and
# with the all-gather exchange (GEOBPE_PEER=0), and the plain one-rank loop beside them; outputs
# under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
K=${2:-"dist_gloo or pipelined_ranks or test_bench"}
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$K" > $OUT/pytest.txt 2>&1; rc=$?
  tail -3 $OUT/pytest.txt
  [ $rc -eq 0 ] || exit $rc
fi
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay"
timeout -k 10 240 $B --steps 20 --warmup 5 > $OUT/bench_window.json 2> $OUT/bench_window.err && echo W_OK && \
timeout -k 10 240 $B --steps 20 --warmup 5 --force-exchange > $OUT/bench_fx_window.json 2> $OUT/bench_fx_window.err && echo FXW_OK && \
GEOBPE_PEER=0 timeout -k 10 240 $B --steps 20 --warmup 5 --force-exchange > $OUT/bench_fxag_window.json 2> $OUT/bench_fxag_window.err && echo FXAGW_OK && \
timeout -k 10 300 $B > $OUT/bench_default.json 2> $OUT/bench_default.err && echo DEF_OK && \
timeout -k 10 300 $B --force-exchange > $OUT/bench_fx_default.json 2> $OUT/bench_fx_default.err && echo FXD_OK && \
GEOBPE_PEER=0 timeout -k 10 300 $B --force-exchange > $OUT/bench_fxag_default.json 2> $OUT/bench_fxag_default.err && echo FXAGD_OK
for f in $OUT/bench_*.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"])' $f 2>/dev/null)"; done
