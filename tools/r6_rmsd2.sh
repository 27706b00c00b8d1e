# usage: bash tools/r6_rmsd2.sh <tag>: the RMSD-mode bench line, the same run with every masked
# re-keying checked by an unmasked one (GEOBPE_REKEY_VERIFY=1), then C5 (merges 11..5000)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --config rmsd --steps 60 --warmup 5 > $OUT/rmsd.out 2> $OUT/rmsd.err && echo RMSD_OK && tail -1 $OUT/rmsd.out && \
GEOBPE_REKEY_VERIFY=1 timeout -k 10 400 python3 bench.py --config rmsd --steps 60 --warmup 5 > $OUT/rmsd_verify.out 2> $OUT/rmsd_verify.err && echo VERIFY_OK && \
timeout -k 10 300 python3 bench.py --gpus 1 --config c5 --steps 4990 --warmup 10 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err && echo C5_OK && tail -1 $OUT/bench_c5.json | cut -c1-200
