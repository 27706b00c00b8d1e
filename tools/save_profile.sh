# usage: bash tools/save_profile.sh <tag>   (after tools/prof.sh <tag> ran on the GPU box)
# copies the rocprofv3 stats / summaries of gpurun_out/prof_<tag> into profiles/r1_<tag>/
# and points profiles/pmc_latest.json (bench.py's roofline.traffic source) at it
set -e
TAG=$1
SRC=gpurun_out/prof_$TAG
DST=profiles/r1_$TAG
mkdir -p $DST
cp $SRC/trace/run_kernel_stats.csv $DST/kernel_stats.csv
python tools/prof_summary.py $SRC profiles/pmc_latest.json $DST > $DST/summary.json
python tools/iter_breakdown.py $SRC > $DST/iter_breakdown.txt
grep -h '^{' $SRC/bench_trace.log | tail -1 > $DST/bench_line_under_rocprof.json || true
echo saved $DST
