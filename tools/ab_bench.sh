# usage: bash tools/ab_bench.sh lib1.so lib2.so ...   (GPU box) -- C3 bench line per library variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for lib in "$@"; do
  GEOBPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay > gpurun_out/ab/$(basename $lib).log 2>&1 || exit 1
  echo "$lib $(grep -h '^{' gpurun_out/ab/$(basename $lib).log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
