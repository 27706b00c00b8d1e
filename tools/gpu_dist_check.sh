# usage: bash tools/gpu_dist_check.sh   (on the GPU box, via gpurun)
# multi-rank tests (gloo ranks sharing the one GPU), then the RCCL world-1 rehearsal bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_dist_gloo.py > gpurun_out/pytest_dist.log 2>&1 && echo DIST_OK && \
timeout -k 10 300 python bench.py --force-exchange > gpurun_out/bench_fx.log 2>&1 && echo BENCH_FX_OK
if [ "$1" = "prof" ]; then
  export TMPDIR=/tmp && mkdir -p gpurun_out/prof_fx && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fx/trace -o run -- python3 bench.py --force-exchange > gpurun_out/prof_fx/bench.log 2>&1 && echo PROF_OK
fi
