# RMSD-mode step timing at 2000 chains over 50 steps (round 2's setting) and a host profile of it
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3_c6
mkdir -p $OUT
timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe 2000 40 120 50 0 1 > $OUT/rmsd_timing_2000_50.json 2> $OUT/rmsd_timing_2000_50.err || exit 1
tail -1 $OUT/rmsd_timing_2000_50.json
GEOBPE_PROFILE=1 timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe 2000 40 120 50 0 1 > $OUT/rmsd_prof.json 2> $OUT/rmsd_prof.txt || exit 1
grep -A30 "Ordered by" $OUT/rmsd_prof.txt | head -40
