#!/bin/bash
# Copies into the host pipeline's pinned slots with streaming stores
# (RDC_HOST_NT_COPY=1, default) vs glibc memcpy (0), same build,
# alternating; n = 2 processes on one GPU (tools/host_path.py).
out=${1:-gpurun_out/host_nt_ab}
mkdir -p $out
port=30600
for k in 1 2; do
  for nt in 1 0; do
    for spec in "16777216 30" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_NT_COPY=$nt timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/nt${nt}_$1_try$k.log 2>&1 || exit 1
      echo "nt $nt $1 $(grep -o '"ms_per_call": [0-9.]*' $out/nt${nt}_$1_try$k.log)"
    done
  done
done
