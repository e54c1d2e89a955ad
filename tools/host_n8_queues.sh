#!/bin/bash
# 8 processes on one GPU: host allreduce at 4 KiB and 64 MiB with 4 (default),
# 2 and 1 hardware queues per process.  A constant ~11 ms per call at the
# default would be the hardware scheduler time-slicing more queues than it
# can map at once (a spinning collective waits for a peer whose queue is
# not mapped until the next slice).
out=${1:-gpurun_out/host_n8_queues}
mkdir -p $out
port=31000
for q in 4 2 1; do
  for spec in "4096 200" "67108864 5"; do
    set -- $spec
    port=$((port+1))
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/q${q}_$1.log 2>&1 || exit 1
    echo "q=$q $1 $(grep host_path $out/q${q}_$1.log | cut -c1-220)"
  done
done
