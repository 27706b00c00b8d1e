# k_glue_opt timing, kept build vs the single-precision-trig A/B build (-DGLUE_DEVICE_TRIG)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python tools/glue_timing.py geobpe 64 60 300 > $OUT/t64_f64.json 2>/dev/null || exit $?
GEOBPE_LIB=$PWD/pt-bpe_amd/geobpe/libgeobpe_ab.so timeout -k 10 300 python tools/glue_timing.py geobpe 64 60 300 > $OUT/t64_f32.json 2>/dev/null || exit $?
timeout -k 10 300 python tools/glue_timing.py geobpe 2000 60 300 > $OUT/t2000_f64.json 2>/dev/null || exit $?
GEOBPE_LIB=$PWD/pt-bpe_amd/geobpe/libgeobpe_ab.so timeout -k 10 300 python tools/glue_timing.py geobpe 2000 60 300 > $OUT/t2000_f32.json 2>/dev/null || exit $?
cat $OUT/*.json
