# usage: bash tools/measure.sh <tag>: rocprofv3 kernel trace + FETCH/WRITE passes of the driver
# window (merges 6..25) and of the default run (merges 11..1000), then tools/fx.sh (multi-rank
# tests, the RCCL rehearsal of the N > 1 loop and its trace); outputs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
( while true; do date +%T >> gpurun_out/heartbeat_$1; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
mkdir -p gpurun_out
bash tools/prof_window.sh $1_w --gpus 1 --steps 20 --warmup 5 || exit 1
bash tools/prof_window.sh $1_d --gpus 1 || exit 1
bash tools/fx.sh $1_fx
