#!/bin/bash
# tools/pcie_duplex.cpp: one process, then two processes started together on
# the same GPU, 64 MiB and 256 MiB.
out=${1:-gpurun_out/pcie_duplex}
mkdir -p $out
for S in 67108864 268435456; do
  timeout -k 10 120 tools/pcie_duplex $S > $out/one_proc_$S.json || exit 1
  t=$(python -c 'import time; print(int(time.time()*1000) + 3000)')
  timeout -k 10 120 tools/pcie_duplex $S $t > $out/two_proc_a_$S.json &
  p=$!
  timeout -k 10 120 tools/pcie_duplex $S $t > $out/two_proc_b_$S.json || exit 1
  wait $p || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(cat $f)"; done
