#!/bin/bash
# Host pipeline copy threads per rank (RDC_HOST_THREADS: pool + caller),
# same build, alternating; n = 2 processes on one GPU (tools/host_path.py).
out=${1:-gpurun_out/host_threads}
mkdir -p $out
port=30700
for k in 1 2; do
  for th in 2 4 6 8; do
    for spec in "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_THREADS=$th timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/t${th}_$1_try$k.log 2>&1 || exit 1
      echo "threads $th $1 $(grep -o '"ms_per_call": [0-9.]*' $out/t${th}_$1_try$k.log)"
    done
  done
done
