# usage: bash tools/r6_s3.sh <tag>: the whole GPU suite, smoke and bench lines (tools/gpu_suite.sh), then
# the driver window with two replica ranks on this one GPU (gloo: both ranks on GPU 0; rank_plan's choice at 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_suite.sh $1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-replay --no-cpu-baseline \
  > gpurun_out/$1/rep2_w.json 2> gpurun_out/$1/rep2_w.err && echo REP2_OK
for f in bench_driver bench_noprof bench_default rep2_w; do echo "$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["config"]["parallelism"])' gpurun_out/$1/$f.json)"; done
