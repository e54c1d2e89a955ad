#!/bin/bash
# Host-path diagnostics: copy options on this box, then the host allreduce at
# 64 / 256 MiB, n = 2 on one GPU, with the per-piece timeline (RDC_HOST_TRACE).
set -e -o pipefail
out=gpurun_out/r3c
mkdir -p $out
timeout -k 10 120 tools/host_copy_bench $((256<<20)) > $out/host_copy.log 2>&1
for S in 67108864 268435456; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29811 tools/host_path.py $S 8 > $out/host_path_$S.log 2>&1
  RDC_HOST_TRACE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29812 tools/host_path.py $S 3 > $out/host_trace_$S.log 2>&1
done
echo done
