# cfg5 shape (1024 x 1 MiB fp32 buckets) with N ranks as processes on ONE GPU:
# one coalesced call vs 1024 separate calls per step.  usage: bash tools/cfg5_compare.sh N [buckets] [bytes]
N=${1:-2}; K=${2:-1024}; B=${3:-1073741824}
port=$((29900 + N))
for mode in "" "--unfused"; do
  port=$((port+10))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
     --master-port $port bench.py --gpus $N --bytes $B --buckets $K --steps 5 --warmup 2 $mode 2>&1 | grep '^{' \
     | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('n=%d %s  %.3f ms/step  algbw %.1f GB/s busbw %.1f GB/s' % (d['n_gpus'], d['config']['workload'], d['ms_per_step'], d['algbw_GBps'], d['busbw_GBps']))" || exit 1
done
