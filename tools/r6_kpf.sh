# usage: bash tools/r6_kpf.sh <tag>: parity subset, default + window bench, shard rehearsals
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "${K:-c3_1000 or test_gpu_parity or tail or mid or dist_gloo or pipelined_ranks}" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay"
timeout -k 10 200 $B --steps 20 --warmup 5 > $OUT/w.json 2> $OUT/w.err || exit 1
timeout -k 10 300 $B > $OUT/d.json 2> $OUT/d.err || exit 1
for f in w d; do echo "$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' $OUT/$f.json)"; done
MIDS=65536 SHARDS="2 4 8" EXTRA="--force-exchange" GEOBPE_COLLAPSE_AT=4096 bash tools/r6_midsweep.sh $1/fx || exit 1
MIDS=65536 SHARDS="2 4" bash tools/r6_midsweep.sh $1/plain
