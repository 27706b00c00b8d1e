# usage: bash tools/mid_ab.sh <tag> <lib.so> <thresholds...>: the default bench run (merges 11..1000)
# once per middle-regime threshold (GEOBPE_MID); outputs under gpurun_out/ab_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; LIB=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for th in "$@"; do
  GEOBPE_MID=$th GEOBPE_LIB=$PWD/$LIB timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay > $OUT/mid_$th.log 2>&1 || { tail -5 $OUT/mid_$th.log; exit 1; }
  echo "mid $th $(grep -h '^{' $OUT/mid_$th.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"])')"
done
