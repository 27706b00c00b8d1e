# usage: bash tools/r3_gluew.sh <tag>: glue optimisation, one wave per chain (k_glue_wave) vs one
# thread per chain (k_glue_opt, GEOBPE_GLUE_THREAD=1): the glue GPU tests (wave), drift against
# the oracle's optimum on 120 chains (both), glue_opt_all timing at 64 and 2000 chains (both);
# outputs under gpurun_out/r3_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3_$1
mkdir -p $OUT
( while true; do date +%T >> $OUT/heartbeat; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 240 python tools/glue_drift.py device profiles/r3_glue/drift_oracle.npz > $OUT/drift_wave.json 2> $OUT/drift_wave.err || exit 1
cat $OUT/drift_wave.json
GEOBPE_GLUE_THREAD=1 timeout -k 10 240 python tools/glue_drift.py device profiles/r3_glue/drift_oracle.npz > $OUT/drift_thread.json 2> $OUT/drift_thread.err || exit 1
cat $OUT/drift_thread.json
for n in "64 60 300" "2000 60 300"; do
  tag=$(echo $n | cut -d' ' -f1)
  timeout -k 10 240 python tools/glue_timing.py geobpe $n > $OUT/timing_wave_$tag.json 2> $OUT/timing_wave_$tag.err || exit 1
  GEOBPE_GLUE_THREAD=1 timeout -k 10 240 python tools/glue_timing.py geobpe $n > $OUT/timing_thread_$tag.json 2> $OUT/timing_thread_$tag.err || exit 1
  echo "$n wave $(cat $OUT/timing_wave_$tag.json) thread $(cat $OUT/timing_thread_$tag.json)"
done
timeout -k 10 700 python -u -m pytest tests/test_glue.py -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt
exit $rc
