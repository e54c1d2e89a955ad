#!/bin/bash
# Registered host buffers at 64 / 256 MiB, n = 2 on one GPU, alternating:
# pageable, registered, registered with the input DMA at most 2 pieces ahead
# (RDC_HOST_REG_AHEAD=2), registered with 16 MiB pieces; box settings that can
# stall registered (userptr) memory are recorded first.
out=${1:-gpurun_out/host_registered_ab2}
mkdir -p $out
{ echo "numa_balancing: $(cat /proc/sys/kernel/numa_balancing 2>&1)";
  echo "thp: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1)";
  echo "khugepaged defrag: $(cat /sys/kernel/mm/transparent_hugepage/khugepaged/defrag 2>&1)"; } > $out/box.txt
cat $out/box.txt
port=30500
for round in 1 2; do
  for v in pin0 pin1 ahead2 piece16; do
    case $v in
      pin0) envs="RDC_BENCH_PINNED=0";;
      pin1) envs="RDC_BENCH_PINNED=1";;
      ahead2) envs="RDC_BENCH_PINNED=1 RDC_HOST_REG_AHEAD=2";;
      piece16) envs="RDC_BENCH_PINNED=1 RDC_HOST_PIECE_BYTES=16M";;
    esac
    for spec in "67108864 20" "268435456 6"; do
      set -- $spec
      port=$((port+1))
      env $envs timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/${v}_$1.r$round.log 2>&1 || exit 1
      echo "$v round=$round $1 $(grep host_path $out/${v}_$1.r$round.log)"
    done
  done
done
