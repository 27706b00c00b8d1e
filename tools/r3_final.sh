# the whole GPU suite, smoke, the driver's bench command (and without events, and the default
# run), the RMSD-mode step timing at 200 / 2000 chains; outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r3_suite.sh $1 || exit 1
OUT=gpurun_out/r3_$1
for n in 200 2000; do
  timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe $n 40 120 50 0 1 > $OUT/rmsd_timing_$n.json 2> $OUT/rmsd_timing_$n.err || exit 1
  tail -1 $OUT/rmsd_timing_$n.json
done
