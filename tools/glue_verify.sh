# glue kernel change check: drift vs the saved reference optimum (must equal the previous
# build's numbers), timing, glue tests
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python tools/glue_drift.py device profiles/r2_glue/drift_oracle.npz > $OUT/drift.json 2> $OUT/drift.err || exit $?
cat $OUT/drift.json
timeout -k 10 300 python tools/glue_timing.py geobpe 64 60 300 > $OUT/glue_timing_64.json 2> $OUT/t64.err || exit $?
cat $OUT/glue_timing_64.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/glue_prof -o glue -- python3 tools/glue_timing.py geobpe 2000 60 300 > $OUT/glue_timing_2000.json 2> $OUT/t2000.err || exit $?
cat $OUT/glue_timing_2000.json
bash tools/glue_gpu.sh $1
