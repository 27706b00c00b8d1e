# glue-opt device tests first; the end-of-round check only if they ended normally
# (pass, or plain test failures: rc 0 / 1), never after a fault, abort or time limit
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$1
timeout -k 10 240 python -u -m pytest tests/test_glue.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/$1/glue_gpu.log 2>&1
rc=$?
echo "glue rc=$rc"
tail -15 gpurun_out/$1/glue_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r2_end.sh $1
