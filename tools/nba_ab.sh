# usage: bash tools/nba_ab.sh "<bench args>" nba1 nba2 ...  (GPU box): the window bench per GEOBPE_NBA value
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nba
ARGS=$1; shift
for v in "$@"; do
  GEOBPE_NBA=$v timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/nba/nba_$v.log 2>&1 || exit 1
  echo "NBA=$v $ARGS $(grep -h '^{' gpurun_out/nba/nba_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v["avg_us"] for k, v in d["kernels"].items()})')"
done
