#!/bin/bash
# Do the host path's copy streams share hardware queues with the collective's
# stream?  n = 2 on one GPU, pageable and registered buffers, with the default
# GPU_MAX_HW_QUEUES (4), with 8, and with the copy streams on queues of their
# own (RDC_HOST_OWN_QUEUES=1), alternating; then traced runs with own queues.
out=${1:-gpurun_out/host_hwq_ab}
mkdir -p $out
port=30800
for round in 1 2; do
  for q in 4 8 own; do
    for pin in 0 1; do
      for spec in "67108864 20" "268435456 6"; do
        set -- $spec
        port=$((port+1))
        hwq=$q; own=0; [ $q = own ] && { hwq=4; own=1; }
        GPU_MAX_HW_QUEUES=$hwq RDC_HOST_OWN_QUEUES=$own RDC_BENCH_PINNED=$pin timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 \
          > $out/q${q}_pin${pin}_$1.r$round.log 2>&1 || exit 1
        echo "q=$q pin=$pin round=$round $1 $(grep host_path $out/q${q}_pin${pin}_$1.r$round.log | cut -c1-200)"
      done
    done
  done
done
RDC_HOST_OWN_QUEUES=1 bash tools/host_registered_trace.sh $out/trace_own || exit 1
