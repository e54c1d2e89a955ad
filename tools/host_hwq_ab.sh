#!/bin/bash
# Do the host path's copy streams share hardware queues with the collective's
# stream?  n = 2 on one GPU, pageable and registered buffers, with the default
# GPU_MAX_HW_QUEUES (4) and with 8, alternating; then one traced run with 8.
out=${1:-gpurun_out/host_hwq_ab}
mkdir -p $out
port=30800
for round in 1 2; do
  for q in 4 8; do
    for pin in 0 1; do
      for spec in "67108864 20" "268435456 6"; do
        set -- $spec
        port=$((port+1))
        GPU_MAX_HW_QUEUES=$q RDC_BENCH_PINNED=$pin timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 \
          > $out/q${q}_pin${pin}_$1.r$round.log 2>&1 || exit 1
        echo "q=$q pin=$pin round=$round $1 $(grep host_path $out/q${q}_pin${pin}_$1.r$round.log | cut -c1-200)"
      done
    done
  done
done
GPU_MAX_HW_QUEUES=8 bash tools/host_registered_trace.sh $out/trace_q8 || exit 1
