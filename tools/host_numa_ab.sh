#!/bin/bash
# Host-buffer allreduce with the whole job confined to the GPU's NUMA node
# (near), to the other node (far), or unconfined; n = 2 processes on one GPU
# (tools/host_path.py), alternating.  The node comes from sysfs.
out=${1:-gpurun_out/host_numa_ab}
mkdir -p $out
# the visible GPU's own CPUs (its render device's local_cpulist, as the
# launcher's --numa-bind reads them) and the rest; /sys/class/drm/card0 is not
# necessarily this box's GPU (the first version of this script read it and
# labelled the two nodes the wrong way round on a box whose GPU is on node 1)
read near far < <(python3 -c "
import os, sys
sys.path.insert(0, '.')
from rdc_amd.launcher import gpu_local_cpus
c = gpu_local_cpus(0)
if not c:
    sys.exit('no GPU-local CPU list')
rest = sorted(os.sched_getaffinity(0) - c)
fmt = lambda s: ','.join(map(str, sorted(s)))
print(fmt(c), fmt(rest))
") || exit 1
echo "gpu-local cpus $near | others $far"
port=31300
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
