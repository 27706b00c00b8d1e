# one GPU call: A/B of the EHASH check's placement (k_find's start vs k_place), the merge-loop
# GPU tests with the check in k_place, then the glue wave-kernel checks (tools/r3_gluew.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r3_ab.sh chk pt-bpe_amd/geobpe/ab_chk0.so pt-bpe_amd/geobpe/ab_chk1.so > gpurun_out/ab_chk.txt 2>&1 || { cat gpurun_out/ab_chk.txt; exit 1; }
cat gpurun_out/ab_chk.txt
GEOBPE_LIB=$PWD/pt-bpe_amd/geobpe/ab_chk1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_tail.py tests/test_c3_parity.py -m gpu -x -q --timeout 600 --timeout-method thread -k "not world8" > gpurun_out/chk1_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/chk1_tests.txt
[ $rc -le 1 ] || exit $rc
bash tools/r3_gluew.sh gw2
