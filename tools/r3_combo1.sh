# one GPU call: kernel A/B of the token rewrites' placement (k_commit vs k_place), the
# switch-batch prediction A/B, then the glue wave-kernel checks (tools/r3_gluew.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r3_ab.sh ct pt-bpe_amd/geobpe/ab_ct0.so pt-bpe_amd/geobpe/ab_ct1.so > gpurun_out/ab_ct.txt 2>&1 || { cat gpurun_out/ab_ct.txt; exit 1; }
cat gpurun_out/ab_ct.txt
bash tools/env_ab.sh swp GEOBPE_SWITCH_PRED "--steps 20 --warmup 5" 0 1 > gpurun_out/ab_swp_w.txt 2>&1 || exit 1
bash tools/env_ab.sh swpd GEOBPE_SWITCH_PRED "" 0 1 > gpurun_out/ab_swp_d.txt 2>&1 || exit 1
cat gpurun_out/ab_swp_w.txt gpurun_out/ab_swp_d.txt | cut -c1-200
bash tools/r3_gluew.sh gw1
