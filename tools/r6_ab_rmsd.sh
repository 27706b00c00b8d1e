# usage: bash tools/r6_ab_rmsd.sh <tag>: round 5's final library against this tree's (tools/r5_step.sh),
# then the RMSD-mode bench line (README downstream setting, 2 000 chains)
set -o pipefail
cd $GRAFT_REPO_ROOT
PYTEST_K="c3_1000 or test_gpu_parity" bash tools/r5_step.sh $1 pt-bpe_amd/geobpe/ab_r5.so pt-bpe_amd/geobpe/ab_r6.so || exit 1
timeout -k 10 600 python3 bench.py --config rmsd --steps 60 --warmup 5 > gpurun_out/$1/rmsd.out 2> gpurun_out/$1/rmsd.err && echo RMSD_OK
tail -1 gpurun_out/$1/rmsd.out
