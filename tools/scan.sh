# per-call allreduce time vs size, n ranks as processes on ONE GPU (protocol + launch cost, not xGMI)
# usage: bash tools/scan.sh N "sizes..." [algo]
N=$1; SIZES=$2; ALGO=${3:-auto}
port=$((29800 + N))
for S in $SIZES; do
  port=$((port+10))
  steps=200; [ $S -ge 67108864 ] && steps=20
  RDC_NBLOCKS=${RDC_NBLOCKS:-64} timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
     --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --bytes $S --steps $steps --warmup 10 --algo $ALGO 2>&1 \
     | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('n=%d S=%10d algo=%s  %.1f us/call  algbw %.1f GB/s' % (d['n_gpus'], d['config']['bytes_per_gpu'], '$ALGO', d['roofline']['kernel_avg_ms']*1e3, d['algbw_GBps']))"
done
