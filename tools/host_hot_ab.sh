#!/bin/bash
# Host pipeline copy threads spinning between pieces (RDC_HOST_POOL_HOT=1,
# default) vs sleeping (0), same build, alternating; n = 2 processes on one
# GPU (tools/host_path.py); then one traced 64 MiB run of each.
out=${1:-gpurun_out/host_hot_ab}
mkdir -p $out
port=31100
for k in 1 2 3; do
  for hot in 1 0; do
    for spec in "33554432 20" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_POOL_HOT=$hot timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/hot${hot}_$1_try$k.log 2>&1 || exit 1
      echo "hot $hot $1 $(grep -o '"ms_per_call": [0-9.]*' $out/hot${hot}_$1_try$k.log)"
    done
  done
done
for hot in 1 0; do
  port=$((port+1))
  RDC_HOST_TRACE=1 RDC_HOST_POOL_HOT=$hot timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/host_path.py 67108864 3 \
    > $out/trace_hot${hot}_67108864.log 2>&1 || exit 1
done
