#!/bin/bash
# A/B of the host-buffer pipeline above 16 MiB (tools/host_path.py, n = 2
# processes on one GPU): ab_old/librdc_amd.so (pageable D2H from a drain
# thread) vs ab_old/librdc_amd_new.so (D2H into pinned output slots, copy-out
# by a pool), alternated on one box; then one traced call of the new build.
# (Round 3, second A/B: old = slices of every chunk per piece, new = contiguous pieces.)
out=${1:-gpurun_out/ab_host_big}
mkdir -p $out
port=30200
for v in new old new old; do
  if [ $v = new ]; then cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so; else cp ab_old/librdc_amd.so rdc_amd/librdc_amd.so; fi
  for spec in "33554432 20" "67108864 12" "268435456 5"; do
    set -- $spec
    port=$((port+1))
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port tools/host_path.py $1 $2 > $out/${v}_$1.$port.log 2>&1 || exit 1
    echo "$v $1 $(grep host_path $out/${v}_$1.$port.log)"
  done
done
cp ab_old/librdc_amd_new.so rdc_amd/librdc_amd.so
RDC_HOST_TRACE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 30299 tools/host_path.py 67108864 3 > $out/trace_new_67108864.log 2>&1
