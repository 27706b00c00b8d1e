# glue-opt device tests only (verbose, every test even after a failure)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_glue.py -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/glue_gpu.log 2>&1
rc=$?
echo "glue rc=$rc"
grep -E "max \\||PASS|FAIL|Error|assert" gpurun_out/$1/glue_gpu.log | head -40
exit $rc
