# usage: bash tools/r6_prof_s3.sh <tag>: rocprofv3 kernel trace + FETCH / WRITE passes of the driver window
# and of merges 11..1000 (tools/prof_window.sh), the C5 bench and the 1/8 share's exchange rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
bash tools/prof_window.sh $1_w --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/prof_window.sh $1_d --gpus 1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --config c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err && echo C5_OK && \
timeout -k 10 200 python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 --force-exchange --shard-of 8 > $OUT/fx_w8.json 2> $OUT/fx_w8.err && echo FX8_OK && \
timeout -k 10 200 python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 --force-exchange > $OUT/fx_w.json 2> $OUT/fx_w.err && echo FX_OK
