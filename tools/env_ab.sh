# usage: bash tools/env_ab.sh <tag> <VAR> "<bench args>" value1 value2 ...   (GPU box)
# one bench line per value of the environment variable VAR (e.g. GEOBPE_MID), outputs under
# gpurun_out/ab_<tag>/; stops at the first failing run
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; ARGS=$3; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay $ARGS > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "$VAR=$v $ARGS $(grep -h '^{' $OUT/$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("kernels"))')"
done
