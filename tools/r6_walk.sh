# usage: bash tools/r6_walk.sh <tag>: C3 parity + gpu parity tests, then the plain window / default bench
# and the shard-of-8 loopback rehearsal trace (outputs under gpurun_out/<tag>/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "${2:-c3_1000 or test_gpu_parity}" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile"
timeout -k 10 200 $B --steps 20 --warmup 5 > $OUT/w.json 2> $OUT/w.err || exit 1
timeout -k 10 300 $B > $OUT/d.json 2> $OUT/d.err || exit 1
GEOBPE_COLLAPSE_AT=4096 timeout -k 10 200 $B --steps 20 --warmup 5 --force-exchange --shard-of 8 > $OUT/lb_w8.json 2> $OUT/lb_w8.err || exit 1
for f in w d lb_w8; do echo "$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' $OUT/$f.json)"; done
GEOBPE_COLLAPSE_AT=4096 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr8 -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 --force-exchange --shard-of 8 > $OUT/tr8.json 2> $OUT/tr8.err && echo TR8_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trd -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile > $OUT/trd.json 2> $OUT/trd.err && echo TRD_OK
