# usage: bash tools/r6_midsweep.sh <tag>: the driver window (merges 6..25) of one rank's share of an
# N-way run (--shard-of N, plain one-rank loop) at several middle-regime thresholds (GEOBPE_MID)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5"
for m in ${MIDS:-65536 32768 16384 8192}; do
  for s in ${SHARDS:-1 2 4 8}; do
    GEOBPE_MID=$m timeout -k 10 200 $B --shard-of $s $EXTRA > $OUT/m${m}_s$s.json 2> $OUT/m${m}_s$s.err || exit 1
    echo "mid $m shard $s $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' $OUT/m${m}_s$s.json)"
  done
done
