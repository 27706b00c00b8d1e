# one GPU call: the place/exchange overlap (GEOBPE_X_OVERLAP 0 vs 1) on the RCCL world-1
# rehearsal (driver window twice, default once), then the multi-rank GPU tests with it on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_xov
for rep in 1 2; do
  for v in 0 1; do
    GEOBPE_X_OVERLAP=$v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --force-exchange > gpurun_out/ab_xov/w$rep.$v.log 2>&1 || { tail -5 gpurun_out/ab_xov/w$rep.$v.log; exit 1; }
    echo "overlap=$v window $(grep -h '^{' gpurun_out/ab_xov/w$rep.$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
for v in 0 1; do
  GEOBPE_X_OVERLAP=$v timeout -k 10 300 python bench.py --gpus 1 --force-exchange > gpurun_out/ab_xov/d.$v.log 2>&1 || { tail -5 gpurun_out/ab_xov/d.$v.log; exit 1; }
  echo "overlap=$v default $(grep -h '^{' gpurun_out/ab_xov/d.$v.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
GEOBPE_X_OVERLAP=1 timeout -k 10 1100 python -u -m pytest tests/test_dist_gloo.py tests/test_bench.py tests/test_c3_parity.py -m gpu -x -v --timeout 1100 --timeout-method thread -k "dist_gloo or test_bench or pipelined_ranks" > gpurun_out/xov_tests.txt 2>&1; rc=$?
tail -4 gpurun_out/xov_tests.txt
exit $rc
