#!/bin/bash
# Custom-reducer allreduce (ICommunicator::Allreduce(Buffer, ReduceFunction)),
# 64 MiB fp32 host buffer, n processes sharing the box's GPU: the round-2
# full-buffer allgather form (custom_reducer_bench_old, built against the
# previous include/rdc.h) vs the chunk exchange (custom_reducer_bench_new),
# alternating.  Binaries are built in the container (tools/Makefile-less:
# g++ -O2 -I include tools/custom_reducer_bench.cc -lrdc_amd).
set -e
n=${1:-4}
mib=${2:-64}
out=${3:-gpurun_out/custom_reducer}
mkdir -p "$out"
for k in 1 2; do
  for v in old new; do
    timeout -k 10 180 python -m rdc_amd.launcher -n "$n" --gpus 1 tools/custom_reducer_bench_$v "$mib" 5 \
        RDC_SCRATCH_BYTES=256M > "$out/${v}_n${n}_${mib}MiB_try$k.jsonl"
  done
done
