#!/bin/bash
# The host pipeline's copies alone (tools/pcie_pipeline_bench.cpp), one
# process, then two processes started together on the same GPU (the n = 2
# rehearsal's sharing), then the real host allreduce at n = 2 for comparison.
out=${1:-gpurun_out/pcie_two_proc}
mkdir -p $out
for S in 67108864 268435456; do
  timeout -k 10 120 tools/pcie_pipeline_bench $S 8388608 10 > $out/one_proc_$S.json || exit 1
  t=$(python -c 'import time; print(int(time.time()*1000) + 3000)')
  timeout -k 10 120 tools/pcie_pipeline_bench $S 8388608 10 $t > $out/two_proc_a_$S.json &
  p=$!
  timeout -k 10 120 tools/pcie_pipeline_bench $S 8388608 10 $t > $out/two_proc_b_$S.json || exit 1
  wait $p || exit 1
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 30400 tools/host_path.py $S 10 > $out/host_path_n2_$S.log 2>&1 || exit 1
done
grep -h . $out/*.json; grep -h host_path $out/host_path_n2_*.log
