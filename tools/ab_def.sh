# usage: bash tools/ab_def.sh <tag> lib1.so lib2.so ...   (GPU box)
# middle-regime A/B: the default bench run (merges 11..1000) three times per library, alternating;
# outputs under gpurun_out/ab_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in "$@"; do
    GEOBPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay > $OUT/$(basename $lib).d$rep.log 2>&1 \
      || { tail -5 $OUT/$(basename $lib).d$rep.log; exit 1; }
    echo "$(basename $lib) d$rep $(grep -h '^{' $OUT/$(basename $lib).d$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel"], d["roofline"].get("avg_launch_us"))')"
  done
done
