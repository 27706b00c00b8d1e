# usage: bash tools/ab.sh <tag> lib1.so lib2.so ...   (GPU box)
# kernel A/B: the driver window (merges 6..25) twice and the default run (merges 11..1000) once
# per library variant, alternating variants; outputs under gpurun_out/ab_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
run() {  # lib, label, bench args...
  local lib=$1 lab=$2; shift 2
  GEOBPE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-replay "$@" > $OUT/$(basename $lib).$lab.log 2>&1 \
    || { tail -5 $OUT/$(basename $lib).$lab.log; exit 1; }
  echo "$(basename $lib) $lab $(grep -h '^{' $OUT/$(basename $lib).$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r={k:(v or {}).get("avg_launch_us") for k,v in [("roof",d.get("roofline"))]+list((d.get("roofline_other") or {}).items())}; print(d["value"], r)')"
}
for rep in 1 2; do
  for lib in "$@"; do run $lib w$rep --steps 20 --warmup 5; done
done
for lib in "$@"; do run $lib def; done
