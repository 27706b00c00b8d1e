# the whole GPU suite, smoke, the driver's bench command (and without events, and the default
# run), the RMSD-mode step timing (200 chains x 20 / 50 steps, 2000 x 50) and glue_opt_all at
# 2000 chains; outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r3_suite.sh $1 || exit 1
OUT=gpurun_out/r3_$1
for a in "200 20" "200 50" "2000 50"; do
  set -- $a
  timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe $1 40 120 $2 0 1 > $OUT/rmsd_timing_$1x$2.json 2> $OUT/rmsd_timing_$1x$2.err || exit 1
  tail -1 $OUT/rmsd_timing_$1x$2.json
done
timeout -k 10 300 python tools/glue_timing.py geobpe 2000 60 300 > $OUT/glue_timing_2000.json 2> $OUT/glue_timing_2000.err && tail -1 $OUT/glue_timing_2000.json
