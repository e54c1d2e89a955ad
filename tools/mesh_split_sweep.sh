# mesh role split (RDC_MESH_SPLIT = scatter,reduce sixteenths; gather the rest), 1 GiB fp32,
# 2 ranks as processes on ONE GPU, grid 256 and 512 blocks; prints ms and role end times
cd $GRAFT_REPO_ROOT
port=29950
for nb in 256 512; do
  for sp in 6,6 4,8 4,10 3,10 5,8 6,8 2,12; do
    port=$((port+3))
    RDC_NBLOCKS=$nb RDC_MESH_SPLIT=$sp timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 10 --warmup 3 --ring-steps 0 --extra-steps 0 \
      --rccl-steps 0 2>&1 | grep '^{' | python -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d['role_timeline']
print('nb=$nb split=$sp %.3f ms  ends: scatter %.0f reduce %.0f gather %.0f us' % (d['ms_per_step'], r['scatter_us']['last_end'], r['reduce_us']['last_end'], r['gather_us']['last_end']))" || exit 1
  done
done
