# mesh schedule, 1 GiB fp32, 2 ranks as processes on ONE GPU: blocks x tile sweep
cd $GRAFT_REPO_ROOT
port=29800
for nb in 128 256 512; do
  for tile in 0 256K 1M; do
    port=$((port+3))
    RDC_NBLOCKS=$nb RDC_TILE_BYTES=$tile timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
       --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 --ring-steps 0 2>&1 | grep '^{' \
       | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('nblocks=$nb tile=$tile %.3f ms/step' % d['ms_per_step'])" || exit 1
  done
done
