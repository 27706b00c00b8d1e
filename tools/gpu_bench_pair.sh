# usage: bash tools/gpu_bench_pair.sh   (on the GPU box, via gpurun)
# GPU parity suite, then the C3 bench line and the C5 (bins {1: 5}, 5000 merges) line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 && echo BENCH_OK && \
timeout -k 10 300 python bench.py --config c5 --steps 4990 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 && echo BENCH_C5_OK
if [ "$1" = "probe" ]; then
  timeout -k 10 300 python tools/debug/select_probe.py 100000 5000 > gpurun_out/select_probe.log 2>&1 && echo PROBE_OK
fi
