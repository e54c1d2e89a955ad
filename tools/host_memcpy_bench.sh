#!/bin/bash
# tools/host_memcpy_bench on the GPU box: one process; two at once; one on the GPU's NUMA node.
out=${1:-gpurun_out/host_memcpy}
mkdir -p $out
node=$(cat /sys/class/drm/card0/device/numa_node 2>/dev/null || echo 0)
near=$(cat /sys/devices/system/node/node$node/cpulist)
for S in 67108864 268435456; do
  timeout -k 10 120 tools/host_memcpy_bench $S > $out/one_$S.json || exit 1
  timeout -k 10 120 tools/host_memcpy_bench $S > $out/two_a_$S.json &
  p=$!
  timeout -k 10 120 tools/host_memcpy_bench $S > $out/two_b_$S.json || exit 1
  wait $p || exit 1
  timeout -k 10 120 taskset -c $near tools/host_memcpy_bench $S > $out/near_$S.json || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(cat $f)"; done
