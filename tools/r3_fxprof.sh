set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3_fxprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_fxprof/p -o run -- python3 bench.py --gpus 1 --force-exchange > gpurun_out/r3_fxprof/bench.json 2> gpurun_out/r3_fxprof/bench.err && echo PROF_OK
