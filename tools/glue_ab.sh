# glue optimiser drift vs the reference's optimiser, both trig builds (A/B), then the glue tests
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python tools/glue_drift.py device profiles/r2_glue/drift_oracle.npz > $OUT/drift_f64trig.json 2> $OUT/drift.err || exit $?
cat $OUT/drift_f64trig.json
GEOBPE_LIB=$PWD/pt-bpe_amd/geobpe/libgeobpe_ab.so timeout -k 10 200 python tools/glue_drift.py device profiles/r2_glue/drift_oracle.npz > $OUT/drift_devtrig.json 2>> $OUT/drift.err || exit $?
cat $OUT/drift_devtrig.json
bash tools/glue_gpu.sh $1
