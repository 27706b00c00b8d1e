# parity file under two library builds (A/B of a host/kernel variant)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abp
for lib in "$@"; do
  GEOBPE_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/abp/$(basename $lib).log 2>&1
  echo "$lib rc=$? $(tail -1 gpurun_out/abp/$(basename $lib).log)"
done
