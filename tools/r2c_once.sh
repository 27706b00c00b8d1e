set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2c/bench_driver.log 2>&1 && echo BENCH_OK && grep '^{' gpurun_out/r2c/bench_driver.log | cut -c1-300 && \
bash tools/prof_window.sh r2c --gpus 1 --steps 20 --warmup 5
