# one GPU call: hot-list threshold A/B (THETA_DIV_BIG 2 vs 8), the merge-loop GPU tests at the
# default (8), the glue GPU tests with their statistics, the device glue golden
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r3_ab.sh theta pt-bpe_amd/geobpe/ab_th2.so pt-bpe_amd/geobpe/ab_th8.so > gpurun_out/ab_theta.txt 2>&1 || { cat gpurun_out/ab_theta.txt; exit 1; }
cat gpurun_out/ab_theta.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_tail.py tests/test_c3_parity.py tests/test_bpe_api.py -m gpu -x -q --timeout 600 --timeout-method thread -k "not world8" > gpurun_out/theta8_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/theta8_tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_glue.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/glue_v1_tests.txt 2>&1; rc=$?
grep -E "glues in another bin|max \||shares|same_bin|PASS|FAIL" gpurun_out/glue_v1_tests.txt | cut -c1-250
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tests/golden/make_device_glue_golden.py gpurun_out/gl_device_golden.json > gpurun_out/dev_golden.log 2>&1; tail -2 gpurun_out/dev_golden.log
