# usage: bash tools/debug/pmc_lds.sh <tag>   (GPU box) -- one SQ PMC pass of the driver-window bench:
# wave cycles split into issue / wait / LDS-issue stalls, LDS cycles and bank conflicts, per
# dispatch (what bounds the pair-count kernel k_bin_count); outputs under gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- \
  python3 bench.py --no-cpu-baseline --no-replay --no-profile --steps 2 --warmup 1 > $OUT/bench.log 2>&1 && echo SQ_OK
