# the RMSD-mode GPU tests, step timing (200 x 20 / 50, 2000 x 50) and a host profile of the
# 2000-chain steps; outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
OUT=gpurun_out/r3_$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rmsd_mode.py tests/test_recover.py tests/test_glue.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for a in "200 20" "200 50" "2000 50"; do
  set -- $a
  timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe $1 40 120 $2 0 1 > $OUT/rmsd_timing_$1x$2.json 2> $OUT/rmsd_timing_$1x$2.err || exit 1
  tail -1 $OUT/rmsd_timing_$1x$2.json
done
GEOBPE_PROFILE=1 timeout -k 10 400 python tools/rmsd_mode_timing.py geobpe 2000 40 120 50 0 1 > $OUT/rmsd_prof.json 2> $OUT/rmsd_prof.txt && tail -1 $OUT/rmsd_prof.json
