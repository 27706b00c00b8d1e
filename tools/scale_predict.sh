# usage: bash tools/scale_predict.sh <tag>: the measured phases DESIGN 5's N > 1 prediction is built
# from, on one GPU: for N = 1, 2, 4, 8 the work of ONE rank of an N-way row sharding of C3
# (bench.py --shard-of N: rank 0's 1/N of the chains, alone on the GPU) -- the plain loop (the
# per-rank kernels) and the world-1 rehearsal of the whole N > 1 protocol on that shard
# (--force-exchange, peer exchange; its collapse at the N-way run's per-rank point), on the driver
# window (merges 6..25) and the default run (merges 11..1000); outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile"
for n in 1 2 4 8; do
  S=""; [ $n -gt 1 ] && S="--shard-of $n"
  CA=$((32768 / n))
  timeout -k 10 200 $B $S --steps 20 --warmup 5 > $OUT/plain_w_$n.json 2> $OUT/plain_w_$n.err || exit 1
  timeout -k 10 300 $B $S > $OUT/plain_d_$n.json 2> $OUT/plain_d_$n.err || exit 1
  GEOBPE_COLLAPSE_AT=$CA timeout -k 10 200 $B $S --steps 20 --warmup 5 --force-exchange > $OUT/fx_w_$n.json 2> $OUT/fx_w_$n.err || exit 1
  GEOBPE_COLLAPSE_AT=$CA timeout -k 10 300 $B $S --force-exchange > $OUT/fx_d_$n.json 2> $OUT/fx_d_$n.err || exit 1
  echo "N=$n done"
done
for f in $OUT/*.json; do echo "$(basename $f) $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' $f)"; done | tee $OUT/summary.txt
