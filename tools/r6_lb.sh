set -o pipefail
cd $GRAFT_REPO_ROOT
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-replay --no-profile"
GEOBPE_XTIME=1 timeout -k 10 200 $B --steps 20 --warmup 5 --force-exchange > gpurun_out/lb_w.json 2> gpurun_out/lb_w.err || exit 1
GEOBPE_XTIME=1 GEOBPE_PEER_LOOPBACK=0 timeout -k 10 200 $B --steps 20 --warmup 5 --force-exchange > gpurun_out/nolb_w.json 2> gpurun_out/nolb_w.err || exit 1
timeout -k 10 300 $B --force-exchange > gpurun_out/lb_d.json 2> gpurun_out/lb_d.err || exit 1
GEOBPE_COLLAPSE_AT=4096 timeout -k 10 200 $B --steps 20 --warmup 5 --force-exchange --shard-of 8 > gpurun_out/lb_w8.json 2> gpurun_out/lb_w8.err || exit 1
GEOBPE_COLLAPSE_AT=4096 timeout -k 10 300 $B --force-exchange --shard-of 8 > gpurun_out/lb_d8.json 2> gpurun_out/lb_d8.err || exit 1
grep xtime gpurun_out/lb_w.err | tail -5; grep xtime gpurun_out/nolb_w.err | tail -5
for f in lb_w nolb_w lb_d lb_w8 lb_d8; do echo "$f $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["config"].get("exchange"))' gpurun_out/$f.json)"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "dist_gloo" > gpurun_out/lb_pytest.txt 2>&1; tail -2 gpurun_out/lb_pytest.txt
