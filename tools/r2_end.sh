# end-of-round check on one MI355X: full GPU suite, smoke(), the driver's bench line, the
# default and exchange-rehearsal benches, then the window profile (trace + FETCH/WRITE passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo SMOKE_OK || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1 && echo DEFAULT_OK || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 && echo BENCH_OK || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --force-exchange > $OUT/bench_fx_window.log 2>&1 && echo FX_OK || exit 1
bash tools/prof_window.sh $1 --gpus 1 --steps 20 --warmup 5
