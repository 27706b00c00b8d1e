# usage: bash tools/r6_final.sh <tag>: the whole GPU suite, smoke and the bench lines (tools/gpu_suite.sh),
# then the world-1 rehearsal of the exchange on the window and the 1/8 share's
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_suite.sh $1 || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5"
timeout -k 10 200 $B --force-exchange > gpurun_out/$1/fx_w.json 2> gpurun_out/$1/fx_w.err && \
timeout -k 10 200 $B --force-exchange --shard-of 8 > gpurun_out/$1/fx_w8.json 2> gpurun_out/$1/fx_w8.err && \
timeout -k 10 200 $B --force-exchange --shard-of 4 > gpurun_out/$1/fx_w4.json 2> gpurun_out/$1/fx_w4.err && \
timeout -k 10 200 $B --force-exchange --shard-of 2 > gpurun_out/$1/fx_w2.json 2> gpurun_out/$1/fx_w2.err || exit 1
for f in bench_driver bench_noprof bench_default fx_w fx_w8 fx_w4 fx_w2; do echo "$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' gpurun_out/$1/$f.json)"; done
