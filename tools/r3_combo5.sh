# one GPU call: middle-regime phase timeline, RMSD-mode step timing (200 and 2000 chains) with the
# C pair keys / span packing; outputs under gpurun_out/r3_c5/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3_c5
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python tools/debug/mid_timeline.py 150,300,600,900 16384 > $OUT/mid_timeline.txt 2>&1 || exit 1
for n in 200 2000; do
  timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe $n 40 120 20 0 1 > $OUT/rmsd_timing_$n.json 2> $OUT/rmsd_timing_$n.err || exit 1
  tail -1 $OUT/rmsd_timing_$n.json
done
