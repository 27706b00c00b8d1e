# usage: bash tools/ab_bench.sh "<bench args>" lib1.so lib2.so ...   (GPU box) -- one bench line per library variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
ARGS=$1; shift
for lib in "$@"; do
  GEOBPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay $ARGS > gpurun_out/ab/$(basename $lib).log 2>&1 || exit 1
  echo "$lib $ARGS $(grep -h '^{' gpurun_out/ab/$(basename $lib).log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
