#!/bin/bash
# Host pipeline with 1 / 2 / 3 drain threads (RDC_HOST_DRAINS), same build,
# alternating; n = 2 processes on one GPU (tools/host_path.py).
out=${1:-gpurun_out/host_drains_ab}
mkdir -p $out
port=31200
for k in 1 2 3; do
  for dr in 1 2 3; do
    for spec in "33554432 20" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_DRAINS=$dr timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/dr${dr}_$1_try$k.log 2>&1 || exit 1
      echo "drains $dr $1 $(grep -o '"ms_per_call": [0-9.]*' $out/dr${dr}_$1_try$k.log)"
    done
  done
done
