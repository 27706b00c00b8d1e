# usage: bash tools/r6_xab.sh <tag> <libs...>: the multi-rank GPU tests with the tree's library, then the
# exchange rehearsal (whole corpus, and the 1/8 share) per library, alternating, twice
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "dist_gloo or pipelined_ranks or collapse" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
[ $rc -eq 0 ] || exit $rc
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 --force-exchange"
for r in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    GEOBPE_LIB=$PWD/$lib timeout -k 10 200 $B > $OUT/${n}_w_$r.json 2>/dev/null || exit 1
    GEOBPE_LIB=$PWD/$lib timeout -k 10 200 $B --shard-of 8 > $OUT/${n}_w8_$r.json 2>/dev/null || exit 1
    echo "$n rep $r: $(python3 -c 'import json,sys; print(*[json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sys.argv[1:]])' $OUT/${n}_w_$r.json $OUT/${n}_w8_$r.json)"
  done
done
