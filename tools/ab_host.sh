#!/bin/bash
# A/B of two builds on one box for host-buffer allreduces (tools/host_path.py,
# n = 2 processes on one GPU): ab_old/librdc_amd.so vs ab_old/librdc_amd_new.so.
out=${1:-gpurun_out/ab_host}
mkdir -p $out
port=30100
for v in new old new old; do
  if [ $v = new ]; then cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so; else cp ab_old/librdc_amd.so rdc_amd/librdc_amd.so; fi
  for spec in "1048576 200" "2097152 100" "4194304 100" "8388608 50" "16777216 30" "67108864 10"; do
    set -- $spec
    port=$((port+1))
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port tools/host_path.py $1 $2 > $out/${v}_$1.$port.log 2>&1 || exit 1
    echo "$v $1 $(grep host_path $out/${v}_$1.$port.log)"
  done
done
cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so
