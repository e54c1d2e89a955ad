#!/bin/bash
# Host allreduce, n = 2 processes on one GPU, one build: a pageable numpy
# buffer (copied through pinned slots) vs the same buffer in a registered
# RdcNewBuffer(pinned=1) range (DMA in place), alternating (tools/host_path.py).
out=${1:-gpurun_out/host_registered_ab}
mkdir -p $out
port=30400
for round in 1 2; do
  for pin in 0 1; do
    for spec in "4194304 100" "16777216 30" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_BENCH_PINNED=$pin timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/pin${pin}_$1.r$round.log 2>&1 || exit 1
      echo "pin=$pin round=$round $1 $(grep host_path $out/pin${pin}_$1.r$round.log)"
    done
  done
done
