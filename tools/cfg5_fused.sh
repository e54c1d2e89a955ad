# cfg5 shape (1024 x 1 MiB fp32 buckets), N ranks as processes on ONE GPU:
# coalesced call through the unit-table mesh (RDC_COALESCE_FUSED=1, default)
# vs pack / mesh / unpack through a staging image (=0).  usage: bash tools/cfg5_fused.sh N
N=${1:-2}
port=$((29700 + N))
for fused in 1 0; do
  port=$((port+10))
  RDC_COALESCE_FUSED=$fused timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
     --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --bytes 1073741824 --buckets 1024 \
     --steps 10 --warmup 3 2>&1 | grep '^{' \
     | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('fused=$fused n=%d %s  %.3f ms/step  algbw %.1f GB/s busbw %.1f GB/s' % (d['n_gpus'], d['config']['workload'], d['ms_per_step'], d['algbw_GBps'], d['busbw_GBps']))" || exit 1
done
