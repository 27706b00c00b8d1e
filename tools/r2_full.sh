# full GPU suite, the driver's bench line, and the RCCL world-1 exchange rehearsal (driver window + full run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 && echo BENCH_OK || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --force-exchange > $OUT/bench_fx_window.log 2>&1 && echo FX1_OK || exit 1
timeout -k 10 300 python3 bench.py --force-exchange > $OUT/bench_fx_full.log 2>&1 && echo FX2_OK || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-replay > $OUT/bench_full.log 2>&1 && echo FULL_OK
