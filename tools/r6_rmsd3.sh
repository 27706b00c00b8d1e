# usage: bash tools/r6_rmsd3.sh <tag>: the RMSD mode's host profile with and without the re-keying's
# residue masks (alternating, twice each), then the glue / RMSD-mode GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python3 tools/debug/rmsd_box_profile.py 2000 40 > /dev/null 2> $OUT/mask_$r.txt || exit 1
  timeout -k 10 300 python3 tools/debug/rmsd_box_profile.py 2000 40 --nomask > /dev/null 2> $OUT/nomask_$r.txt || exit 1
done
grep -h "ms a step" $OUT/*.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "glue or rmsd" > $OUT/pytest.txt 2>&1; rc=$?
tail -2 $OUT/pytest.txt
exit $rc
