#!/bin/bash
# Host-buffer allreduce (tools/host_path.py, n = 2 processes on one GPU) by
# pipeline piece size (RDC_HOST_PIECE_BYTES) and buffer size.
out=${1:-gpurun_out/host_piece}
mkdir -p $out
port=30300
for piece in ${PIECES:-16777216 4194304 8388608 33554432}; do
  for spec in "16777216 20" "67108864 8" "268435456 4"; do
    set -- $spec
    port=$((port+1))
    RDC_HOST_PIECE_BYTES=$piece timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/p${piece}_$1.log 2>&1 || exit 1
    echo "piece $piece bytes $1 $(grep -o '"ms_per_call": [0-9.]*' $out/p${piece}_$1.log)"
  done
done
