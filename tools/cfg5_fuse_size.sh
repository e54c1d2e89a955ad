# cfg5 shape (1024 x 1 MiB fp32), 2 ranks as processes on ONE GPU: unit-table
# mesh with fusion groups of RDC_FUSE_BYTES = 64M / 256M / 1G
cd $GRAFT_REPO_ROOT
port=29750
for fb in 64M 256M 1G; do
  port=$((port+10))
  RDC_FUSE_BYTES=$fb timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
     --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --bytes 1073741824 --buckets 1024 \
     --steps 10 --warmup 3 2>&1 | grep '^{' \
     | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('fuse=$fb %.3f ms/step busbw %.1f GB/s' % (d['ms_per_step'], d['busbw_GBps']))" || exit 1
done
