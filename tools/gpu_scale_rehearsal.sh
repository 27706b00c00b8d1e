# usage: bash tools/gpu_scale_rehearsal.sh   (GPU box) -- bench.py's N > 1 code path end to end:
# 2 and 3 ranks (gloo, all on GPU 0) through torch.distributed.run, as the driver launches N > 1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 2 3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 290 --warmup 10 --dist-backend gloo \
    > gpurun_out/scale_$n.log 2>&1 || exit 1
  echo "N=$n $(grep -h '^{' gpurun_out/scale_$n.log | tail -1)"
done
