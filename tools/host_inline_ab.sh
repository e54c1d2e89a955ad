#!/bin/bash
# 2-16 MiB host buffers: one inline piece (default) vs the pipeline with small
# pieces (RDC_HOST_INLINE_BYTES=1M, RDC_HOST_PIECE_BYTES=2M / 1M), same build,
# alternating; n = 2 processes on one GPU (tools/host_path.py).
out=${1:-gpurun_out/host_inline_ab}
mkdir -p $out
port=30800
for k in 1 2; do
  for cfg in "inline 16M 8M" "p2m 1M 2M" "p1m 1M 1M"; do
    set -- $cfg
    name=$1; inl=$2; pc=$3
    for spec in "4194304 60" "8388608 40" "16777216 30"; do
      set -- $spec
      port=$((port+1))
      RDC_HOST_INLINE_BYTES=$inl RDC_HOST_PIECE_BYTES=$pc timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 \
        > $out/${name}_$1_try$k.log 2>&1 || exit 1
      echo "$name $1 $(grep -o '"ms_per_call": [0-9.]*' $out/${name}_$1_try$k.log)"
    done
  done
done
