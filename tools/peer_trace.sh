# usage: bash tools/peer_trace.sh <tag> [bench args]: kernel trace of the world-1 rehearsal of the N > 1 loop
# (--force-exchange) on the driver window, peer exchange and all-gather exchange; window summaries
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p $OUT
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 --force-exchange $*"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/peer -o run -- $B > $OUT/peer.json 2> $OUT/peer.err && echo PEER_OK && \
GEOBPE_PEER=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ag -o run -- $B > $OUT/ag.json 2> $OUT/ag.err && echo AG_OK
python3 tools/trace_window.py $OUT/peer > $OUT/peer_window.txt; python3 tools/trace_window.py $OUT/ag > $OUT/ag_window.txt
cat $OUT/peer_window.txt $OUT/ag_window.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/plain -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile --steps 20 --warmup 5 $* > $OUT/plain.json 2> $OUT/plain.err && echo PLAIN_OK
python3 tools/trace_window.py $OUT/plain > $OUT/plain_window.txt; cat $OUT/plain_window.txt
