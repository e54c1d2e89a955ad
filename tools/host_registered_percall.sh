#!/bin/bash
# Per-call times of registered host buffers (n = 2 on one GPU): which call is slow.
out=${1:-gpurun_out/host_registered_percall}
mkdir -p $out
port=30600
for spec in "pin1 67108864 30" "pin1 268435456 10" "pin0 67108864 30"; do
  set -- $spec
  port=$((port+1))
  p=0; [ $1 = pin1 ] && p=1
  RDC_BENCH_PER_CALL=1 RDC_BENCH_PINNED=$p timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/host_path.py $2 $3 > $out/$1_$2.log 2>&1 || exit 1
  echo "$1 $2 $(grep host_path $out/$1_$2.log)"
done
