#!/bin/bash
# Host path helper threads pinned to the GPU's NUMA node (default) vs left
# to the OS (RDC_HOST_AFFINITY=0), unconfined job, same build, alternating;
# n = 2 processes on one GPU (tools/host_path.py).
out=${1:-gpurun_out/host_affinity_ab}
mkdir -p $out
port=31000
for k in 1 2 3; do
  for aff in 1 0; do
    for spec in "16777216 30" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_AFFINITY=$aff timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/aff${aff}_$1_try$k.log 2>&1 || exit 1
      echo "aff $aff $1 $(grep -o '"ms_per_call": [0-9.]*' $out/aff${aff}_$1_try$k.log)"
    done
  done
done
