# usage: bash tools/debug/rmsd_ab.sh <tag> [rmsdkey variant .so ...] (GPU box): tools/rmsd_mode_timing.py
# (2 000 chains, 50 steps from the first) three times per build, builds alternating (the in-tree
# _rmsdkey.so first, then each variant through GEOBPE_RMSDKEY: host speed drifts on a shared
# machine), then tools/debug/rmsd_host_time.py --warm=0 once each; outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; shift
mkdir -p $OUT
libs=("" "$@")
lab() { [ -z "$1" ] && echo base || basename $1 .so; }
for rep in 1 2 3; do
  for lib in "${libs[@]}"; do
    l=$(lab "$lib")
    GEOBPE_RMSDKEY=${lib:+$PWD/$lib} timeout -k 10 300 python -u tools/rmsd_mode_timing.py geobpe 2000 40 120 50 0 2>$OUT/$l.err | grep '^{' > $OUT/$l.timing$rep.json || exit 1
    echo "$l rep$rep $(python -c "import json; print(round(1000 * json.load(open('$OUT/$l.timing$rep.json'))['s_per_step'], 3))") ms/step"
  done
done
for lib in "${libs[@]}"; do
  l=$(lab "$lib")
  GEOBPE_RMSDKEY=${lib:+$PWD/$lib} timeout -k 10 300 python -u tools/debug/rmsd_host_time.py 2000 40 120 50 --device --warm=0 2>&1 | grep -v Converged > $OUT/$l.host.txt || exit 1
  echo "$l $(head -2 $OUT/$l.host.txt | tail -1)"
done
