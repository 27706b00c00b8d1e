set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_dist_gloo.py tests/test_gpu_parity.py -k "shard or dist or pipelin or gloo or world" > $OUT/pytest.log 2>&1; rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --force-exchange > $OUT/fx_window.log 2>&1 && echo FX1_OK || exit 1
timeout -k 10 300 python3 bench.py --force-exchange > $OUT/fx_full.log 2>&1 && echo FX2_OK
