#!/bin/bash
# cfg5's shape vs one buffer, same box, alternating (N = 2 on one GPU, each
# autotuned for the 1 GiB class); then full N = 4 and N = 8 rehearsals.
set -o pipefail
out=gpurun_out/r3f
mkdir -p $out
fast="--extra-steps 0 --rccl-steps 0 --cpu-seconds 0 --ring-steps 0 --no-check --steps 30"
for k in 1 2; do
  for b in 1 1024; do
    bash tools/gpu_rehearse.sh 2 $out/n2_buckets${b}_try$k.log $fast --buckets $b || exit 1
  done
done
bash tools/gpu_rehearse.sh 4 $out/bench_n4.log || exit 1
bash tools/gpu_rehearse.sh 8 $out/bench_n8.log || exit 1
