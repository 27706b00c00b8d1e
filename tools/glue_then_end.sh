# glue-opt device tests + timing first; the end-of-round check only if they ended normally
# (pass, or plain test failures: rc 0 / 1), never after a fault, abort or time limit
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_glue.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/glue_gpu.log 2>&1
rc=$?
echo "glue rc=$rc"
tail -12 $OUT/glue_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/glue_timing.py geobpe 64 60 300 > $OUT/glue_timing_64.json 2> $OUT/glue_timing_64.err || exit $?
cat $OUT/glue_timing_64.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/glue_prof -o glue -- python3 tools/glue_timing.py geobpe 2000 60 300 > $OUT/glue_timing_2000.json 2> $OUT/glue_timing_2000.err || exit $?
cat $OUT/glue_timing_2000.json
bash tools/r2_end.sh $1
