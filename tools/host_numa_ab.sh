#!/bin/bash
# Host-buffer allreduce with the whole job confined to the GPU's NUMA node
# (near), to the other node (far), or unconfined; n = 2 processes on one GPU
# (tools/host_path.py), alternating.  The node comes from sysfs.
out=${1:-gpurun_out/host_numa_ab}
mkdir -p $out
node=$(cat /sys/class/drm/card0/device/numa_node 2>/dev/null || echo 0)
near=$(cat /sys/devices/system/node/node$node/cpulist)
far=$(cat /sys/devices/system/node/node$((1 - node))/cpulist 2>/dev/null || echo $near)
echo "gpu numa node $node near $near far $far"
port=30900
for k in 1 2; do
  for cfg in "free" "near" "far"; do
    case $cfg in free) pre="";; near) pre="taskset -c $near";; far) pre="taskset -c $far";; esac
    for spec in "16777216 30" "67108864 12" "268435456 5"; do
      set -- $spec
      port=$((port+1))
      $pre timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port $port tools/host_path.py $1 $2 > $out/${cfg}_$1_try$k.log 2>&1 || exit 1
      echo "$cfg $1 $(grep -o '"ms_per_call": [0-9.]*' $out/${cfg}_$1_try$k.log)"
    done
  done
done
