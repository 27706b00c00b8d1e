# usage: bash tools/ab_run.sh "<bench args>" lib1.so lib2.so ...   (GPU box) -- bench value + per-kernel avg per variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
ARGS=$1; shift
for lib in "$@"; do
  GEOBPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/ab/$(basename $lib).log 2>&1 || exit 1
  echo "$lib $ARGS $(grep -h '^{' gpurun_out/ab/$(basename $lib).log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v["avg_us"] for k, v in d["kernels"].items()})')"
done
