# usage: bash tools/ab_env.sh <tag> "VAR=a" "VAR=b" ... (GPU box): the driver window twice and the
# default run once per environment setting, alternating; outputs under gpurun_out/abe_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/abe_$TAG
mkdir -p $OUT
run() {  # env setting, label, bench args...
  local e=$1 lab=$2; shift 2
  local f=$OUT/$(echo "$e" | tr '= ' '__').$lab.log
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "$e $lab $(grep -h '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("roofline") or {}; print(d["value"], r.get("kernel"), r.get("avg_launch_us"), r.get("live_avg_launch_us"))')"
}
for rep in 1 2; do
  for e in "$@"; do run "$e" w$rep --steps 20 --warmup 5; done
done
for e in "$@"; do run "$e" def; done
